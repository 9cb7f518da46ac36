#!/usr/bin/env python3
"""Instruction mix of a kernel's loops in a hipcc -save-temps .s file.
usage: asm_loop_stats.py file.s mangled_kernel_name"""
import collections
import re
import sys

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
    if m:
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            loops.append((labels[tgt], i))
print(f"{name}: {len(body)} lines, {len(loops)} back-edges")
for s, e in sorted(loops, key=lambda x: x[0] - x[1])[:3]:
    c = collections.Counter()
    for l in body[s:e + 1]:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        c[t.split()[0]] += 1
    tot = sum(c.values())
    print(f"  loop lines {s}-{e}: {tot} instructions")
    for k, v in c.most_common(14):
        print(f"    {v:6d} {k}")
