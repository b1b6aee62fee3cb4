"""Debug: per-op determinism under 4 concurrent streams (WNSA ops at 64x64, B=2, fp16)."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from lic_amd.model import net_ga
from lic_amd.functional import Act
import lic_amd.functional as Fn

torch.manual_seed(0)
net = net_ga.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False, precision="fp16").to("cuda")
w = net.a_model.transform[8]
cb = w.conv_b
wba = cb[0]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
g = torch.Generator().manual_seed(5)
x = Act((torch.randn(B, 64, 64, 192, generator=g)).to(torch.float16).cuda())
q = wba.attn.qkv.run(x)
a_in = Act((torch.randn(B, 64, 64, 192, generator=g) * 0.5).to(torch.float16).cuda())
ops = {
    "qkv1x1": lambda: wba.attn.qkv.run(x),
    "attn": lambda: Fn.win_attn(q, wba.dim, wba.num_heads, wba.window_size, wba.shift_size,
                                wba.attn.relative_position_bias_table, wba.num_heads, 1, 1, False,
                                float(wba.attn.scale)),
    "proj_r1": lambda: wba.attn.proj.run(a_in, None, r1=x),
    "c1x1": lambda: cb[1].run(x),
    "rb": lambda: cb[3].run(x),
    "c3x3": lambda: cb[4].run(x),
    "c7x7": lambda: cb[7].run(x),
    "gate": lambda: cb[9].run(x, None, gate_a=a_in, gate_r=x),
    "wba_full": lambda: wba.run(x),
}
streams = [torch.cuda.Stream() for _ in range(4)]
NT = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for name, f in ops.items():
    ref = f().t.clone()
    torch.cuda.synchronize()
    bad = 0
    for trial in range(NT):
        main = torch.cuda.current_stream()
        for s in streams:
            s.wait_stream(main)
        outs = []
        for s in streams:
            with torch.cuda.stream(s):
                outs.append([f().t for _ in range(3)])
        for s in streams:
            main.wait_stream(s)
        torch.cuda.synchronize()
        bad += sum(0 if torch.equal(o, ref) else 1 for lst in outs for o in lst)
    print(f"{name:10s} mismatching outputs {bad} / {NT * 12}", flush=True)
