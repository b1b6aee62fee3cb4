"""Debug: run growing prefixes of the analysis transform on 4 concurrent streams
(identical inputs, separate outputs) and report the first layer whose output differs
from the serial run."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from lic_amd.model import net_ga
from lic_amd.functional import Act

torch.manual_seed(0)
net = net_ga.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False, precision="fp16").to("cuda")
t = net.a_model.transform
steps = [("rb0", lambda x: t[0].run(x)), ("rb1", lambda x: t[1].run(x)), ("rb2", lambda x: t[2].run(x)),
         ("rbws3", lambda x: t[3].run(x)), ("gdn4", lambda x: t[4].run(x)),
         ("conv5x5_6", lambda x: t[6].run(x, pad=(1, 1, 2, 2))), ("gdn7", lambda x: t[7].run(x)),
         ("wnsa8", lambda x: t[8].run(x)), ("rb9", lambda x: t[9].run(x)), ("rb10", lambda x: t[10].run(x)),
         ("rb11", lambda x: t[11].run(x)), ("rbws12", lambda x: t[12].run(x)), ("gdn13", lambda x: t[13].run(x)),
         ("conv5x5_15", lambda x: t[15].run(x, pad=(1, 1, 2, 2))), ("wnsa16", lambda x: t[16].run(x))]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
x = (torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(5)) * 2 - 1).to("cuda")
x_act = Act.from_nchw(x, torch.float16, pad16=True)
torch.cuda.synchronize()
# serial reference of every step
ref, cur = [], x_act
for name, f in steps:
    cur = f(cur)
    ref.append(cur.t.clone())
torch.cuda.synchronize()
streams = [torch.cuda.Stream() for _ in range(4)]
for trial in range(6):
    outs = [[] for _ in streams]
    main = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(main)
    for si, s in enumerate(streams):
        with torch.cuda.stream(s):
            cur = x_act
            for name, f in steps:
                cur = f(cur)
                outs[si].append(cur.t)
    for s in streams:
        main.wait_stream(s)
    torch.cuda.synchronize()
    bad = []
    for si in range(4):
        for k, (name, _) in enumerate(steps):
            if not torch.equal(outs[si][k], ref[k]):
                bad.append(f"s{si}:{name}")
                break
    print("trial", trial, bad, flush=True)
