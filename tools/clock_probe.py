#!/usr/bin/env python3
"""Can the bench read the GFX clock of its own GPU while it runs?  amdsmi handles, their
BDFs, torch's PCI ids of cuda:0, and 20 samples of amdsmi_get_clock_info(GFX) (idle, then
under a 65536^2 K1t load)."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import amdsmi  # noqa: E402
import torch  # noqa: E402

t0 = time.perf_counter()
amdsmi.amdsmi_init(amdsmi.AmdSmiInitFlags.INIT_AMD_GPUS)
print("init s", round(time.perf_counter() - t0, 3))
hs = amdsmi.amdsmi_get_processor_handles()
for h in hs:
    print("bdf", amdsmi.amdsmi_get_gpu_device_bdf(h))
p = torch.cuda.get_device_properties(0)
print("torch pci", p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
mine = [h for h in hs if int(amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")[1], 16) == p.pci_bus_id]
print("matched", len(mine))
h = mine[0] if mine else hs[0]
t0 = time.perf_counter()
print("clock", amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX),
      "s", round(time.perf_counter() - t0, 4))
try:
    m = amdsmi.amdsmi_get_gpu_metrics_info(h)
    print("metrics keys", [k for k in m if "clk" in k or "clock" in k])
    print({k: m[k] for k in m if "gfxclk" in k})
except Exception as ex:  # noqa: BLE001
    print("metrics failed", ex)
import gol  # noqa: E402
os.environ["GOL_MULTI_VARIANT"] = "15"
os.environ["GOL_TILE"] = "30,524"
e = gol.Engine(65536, 65536, device=0, band_rows=536, turns_per_launch=20)
e.fill_random(3)
samples = []
stop = False


def poll():
    while not stop:
        samples.append(amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)["clk"])
        time.sleep(0.005)


th = threading.Thread(target=poll)
th.start()
e.step(400)
e.sync()
stop = True
th.join()
print("under load", len(samples), samples[:40])
try:
    m = amdsmi.amdsmi_get_gpu_metrics_info(h)
    print({k: m[k] for k in m if "gfxclk" in k})
except Exception as ex:  # noqa: BLE001
    print("metrics failed", ex)
