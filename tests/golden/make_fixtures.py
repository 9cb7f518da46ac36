"""Generate tests/golden/ from the reference's own data files (run once, in the
build container where /root/reference exists; the outputs are committed).

Copied data (not source):
  Local/images/{16,64,128,256,512}^2.pgm      -> images/<name>.pgm.gz   (inputs)
  Local/check/images/{16,64,512}x*x{0,1,100}   -> check/<name>.pgm.gz    (expected boards)
  Local/check/alive/{16,64,512}.csv            -> alive/<name>.csv.gz    (expected counts)
Digests only:
  Local/out/*.pgm                              -> out_manifest.json      (sha256 of the W*H
                                                  pixel payload + alive count + the turn in
                                                  the file name; see SURVEY.md §4 for why
                                                  many of these names are mislabelled)
"""
import gzip
import hashlib
import json
import os
import shutil
import sys

REF = "/root/reference/Local"
HERE = os.path.dirname(os.path.abspath(__file__))


def payload(path):
    data = open(path, "rb").read()
    # header: P5 <ws> W <ws> H <ws> 255 <single ws> payload (Local/gol/io.go:88-121)
    fields, pos = [], 0
    for _ in range(4):
        while data[pos:pos + 1].isspace():
            pos += 1
        start = pos
        while not data[pos:pos + 1].isspace():
            pos += 1
        fields.append(data[start:pos].decode())
    pos += 1
    w, h = int(fields[1]), int(fields[2])
    return w, h, data[pos:pos + w * h]


def gz_copy(src, dst):
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(src, "rb") as f, gzip.GzipFile(dst, "wb", mtime=0) as g:
        shutil.copyfileobj(f, g)


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present; fixtures are already committed")
    manifest = {"images": {}, "check": {}, "alive": {}}
    for name in sorted(os.listdir(f"{REF}/images")):
        gz_copy(f"{REF}/images/{name}", f"{HERE}/images/{name}.gz")
        w, h, p = payload(f"{REF}/images/{name}")
        manifest["images"][name] = {"sha256": hashlib.sha256(p).hexdigest(),
                                    "alive": sum(1 for b in p if b == 255)}
    for name in sorted(os.listdir(f"{REF}/check/images")):
        gz_copy(f"{REF}/check/images/{name}", f"{HERE}/check/{name}.gz")
        w, h, p = payload(f"{REF}/check/images/{name}")
        manifest["check"][name] = {"sha256": hashlib.sha256(p).hexdigest(),
                                   "alive": sum(1 for b in p if b == 255)}
    for name in sorted(os.listdir(f"{REF}/check/alive")):
        gz_copy(f"{REF}/check/alive/{name}", f"{HERE}/alive/{name}.gz")
        manifest["alive"][name] = {"sha256": hashlib.sha256(
            open(f"{REF}/check/alive/{name}", "rb").read()).hexdigest()}
    out = {}
    for name in sorted(os.listdir(f"{REF}/out")):
        stem = name[:-4]
        parts = stem.split("x")
        if len(parts) != 3:
            continue                       # 16x16.pgm etc: no turn in the name (truncated runs)
        try:
            w, h, p = payload(f"{REF}/out/{name}")
        except Exception:
            continue
        if len(p) != w * h:
            continue
        out[name] = {"width": w, "height": h, "turn_in_name": int(parts[2]),
                     "sha256": hashlib.sha256(p).hexdigest(),
                     "alive": sum(1 for b in p if b == 255)}
    manifest["out"] = out
    with open(f"{HERE}/manifest.json", "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(manifest["images"]), "inputs,", len(manifest["check"]), "checks,",
          len(out), "out digests")


if __name__ == "__main__":
    main()
