#!/usr/bin/env python3
"""Which additions does a bf16 training step issue, by dtype, shape and parent op?  Runs
train_net_unet.py eagerly (1 warm-up + 1 timed step) under torch.profiler (CPU events, shapes) and
prints the add calls of the last step grouped by (parent chain, input shapes)."""
import collections
import os
import runpy
import sys

from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = ["train_net_unet.py", "--bench", "--steps", "1", "--warmup", "1", "--eager"]
with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
    runpy.run_path(os.path.join(ROOT, "train_net_unet.py"), run_name="__main__")
par = collections.Counter()
tot = collections.Counter()
for e in prof.events():
    if e.name in ("aten::add", "aten::add_"):
        p = e.cpu_parent
        chain = []
        while p is not None and len(chain) < 2:
            chain.append(p.name)
            p = p.cpu_parent
        shp = str(e.input_shapes)[:80]
        par[(" <- ".join(chain) or "(top level)", shp)] += 1
        tot[" <- ".join(chain) or "(top level)"] += 1
for k, v in tot.most_common(12):
    print(f"{v:6d}  {k[:160]}")
print("---")
for (k, s), v in par.most_common(60):
    print(f"{v:5d}  {k[:90]:90s} {s}")
