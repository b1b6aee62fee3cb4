#!/usr/bin/env python3
"""Which host-side ops issue the small float additions of a training step?  Runs
train_net_unet.py eagerly (bf16, 1 warm-up + 1 timed step) under torch.profiler (CPU events
only) and counts the parent op of every aten::add / aten::add_ call."""
import collections
import os
import runpy
import sys

from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = ["train_net_unet.py", "--bench", "--steps", "1", "--warmup", "1", "--eager"]
with profile(activities=[ProfilerActivity.CPU]) as prof:
    runpy.run_path(os.path.join(ROOT, "train_net_unet.py"), run_name="__main__")
par = collections.Counter()
for e in prof.events():
    if e.name in ("aten::add", "aten::add_"):
        p = e.cpu_parent
        chain = []
        while p is not None and len(chain) < 3:
            chain.append(p.name)
            p = p.cpu_parent
        par[" <- ".join(chain) or "(top level)"] += 1
for k, v in par.most_common(15):
    print(f"{v:6d}  {k[:200]}")
