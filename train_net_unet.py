#!/usr/bin/env python3
"""train_net_unet.py — the reference training CLI (train_net_unet.py:90-238, BASELINE config 5)
on the liblic training path.

What it does per step, as the reference (:167-200): ``bpp, mse = net(x, 'train')``;
``loss = lambda * 255**2 * mse + bpp``; backward; ``clip_grad_norm_(params, 1)``;
``Adam(base_params)`` step; ``MultiStepLR([1500, 2500, 3500, 4000], 0.5)`` per epoch.

Differences:
  * the model is ``--arch net_unet_ha_hs`` (default; SURVEY.md 2 row 17: the U-Net hyper-prior
    net the script's name refers to) or net_ga (eval_net.py's model): the reference script's
    ``model/Net_unet.py`` imports the missing ``model/Block.py`` and cannot be built;
  * one process per GPU (``torch.distributed.run``) with a bucketed gradient all-reduce
    (lic_amd.distributed.GradAllReduce, RCCL over xGMI) instead of single-process
    ``nn.DataParallel`` (:152): eager steps launch each bucket from a post-accumulate-grad hook
    while the backward continues; a captured step (``--graph``, opt-in at world > 1) launches all
    buckets after the backward (serialised cost);
  * data: no DIV2K and no network here — ``--synthetic`` (default) draws random 256x256
    crops from a seeded bank of smooth synthetic images resident in HBM;
  * ``--precision bf16`` (default, BASELINE config 5): bf16 activations / MFMA operands
    (v_mfma_f32_32x32x16_bf16), fp32 accumulation and fp32 master weights, no loss scale;
    ``fp16`` uses a dynamic loss scale (torch.amp.GradScaler); ``fp32`` is the parity path;
  * the NaN check (:189-190) runs every ``--log_every`` steps instead of syncing each step.

``--bench``: W warm-up + K timed steps between barriers + device syncs; rank 0 prints one
JSON line (images/s of the whole job, MAX step time over ranks).
"""
import argparse
import contextlib
import json
import math
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def synthetic_bank(n, size, seed, device):
    from eval_net import synthetic_image
    return torch.stack([synthetic_image(seed + i, size, size) for i in range(n)]).to(device) * 2 - 1


class Crops:
    """RandomCrop(crop) + Preprocess ([-1, 1]) over an HBM-resident image bank (:24-51)."""

    def __init__(self, bank, batch, crop, seed):
        self.bank, self.batch, self.crop = bank, batch, crop
        self.rng = random.Random(seed)

    def __call__(self):
        n, _, H, W = self.bank.shape
        out = []
        for _ in range(self.batch):
            i = self.rng.randrange(n)
            y, x = self.rng.randrange(H - self.crop + 1), self.rng.randrange(W - self.crop + 1)
            out.append(self.bank[i, :, y:y + self.crop, x:x + self.crop])
        return torch.stack(out).contiguous()


def main():
    ap = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument("--train_data_path", default="", help="unused: no dataset ships; see --synthetic")
    ap.add_argument("--weight_path", default="", help="Path of Pretrained Checkpoint")
    ap.add_argument("--checkpoint_dir", default="", help="Directory of Saved Checkpoints ('' = do not save)")
    ap.add_argument("--high", action="store_true", help="Using High Bitrate Model")
    ap.add_argument("--post_processing", action="store_true", help="Using Post Processing (not trainable yet)")
    ap.add_argument("--lambda", type=float, default=0.0025, dest="lmbda")
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--batch_size", type=float, default=8, help="images per GPU")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="activation dtype (fp32 master weights, fp32 accumulation); bf16 = BASELINE config 5")
    ap.add_argument("--crop", type=int, default=256)
    ap.add_argument("--arch", default="net_unet_ha_hs", choices=["net_unet_ha_hs", "net_ga"])
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--steps_per_epoch", type=int, default=20)
    ap.add_argument("--log_every", type=int, default=10)
    ap.add_argument("--bench", action="store_true", help="time --steps steps after --warmup, print JSON")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without torchrun this process starts them itself")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole step (forward, backward, RCCL gradient all-reduce, clip, Adam) in "
                         "one hipGraph and replay it: no per-launch host cost; the noise seed lives on the device "
                         "(bf16 / fp32, any world size; the default there)")
    ap.add_argument("--eager", action="store_true", help="run every step eagerly (no hipGraph capture)")
    ap.add_argument("--ref-clip", action="store_true",
                    help="the reference's exact clip: gradients of every parameter (the non-optimised slice "
                         "modules' accumulating across steps) in clip_grad_norm_ (train_net_unet.py:198)")
    args = ap.parse_args()

    from lic_amd import distributed as D
    if args.gpus > 1 and not D.launched():
        # one process per GPU, started before this process touches the GPU (no re-exec)
        sys.exit(D.launch_workers([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], args.gpus))
    from lic_amd.model import net_ga, net_unet_ha_hs
    from lic_amd import functional as Fn
    from lic_amd import autograd as AG
    rank, world, local = D.init("nccl")
    if D.launched() and args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"train_net_unet.py: --gpus {args.gpus} but the launcher started {world} ranks")
    # bf16 / fp32 on ONE GPU: the captured step is the default (replays equal the eager steps,
    # tests/test_gpu_train_net.py::test_train_step_hipgraph_matches_eager; ~7000 launches per step
    # otherwise leave the GPU waiting on the host).  At world > 1 it is opt-in (--graph): the captured
    # RCCL all-reduce is tested on one rank only (test_gpu_dist_train.py), no multi-rank captured step
    # has run yet
    args.graph = not args.eager and (args.graph or (world == 1 and args.precision != "fp16"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B = int(args.batch_size)

    torch.manual_seed(0)
    mod = net_ga if args.arch == "net_ga" else net_unet_ha_hs
    net = mod.Net((B, args.crop, args.crop, 3), (1, args.crop, args.crop, 3), args.high, args.post_processing,
                  precision=args.precision)
    if args.weight_path:
        net.load_state_dict(torch.load(args.weight_path, map_location="cpu", weights_only=True), strict=True)
    net = net.to(dev)
    params = net.base_params()
    # The reference optimises base_params() only (train_net_unet.py:132) and its opt.zero_grad() clears
    # only theirs: the slice-loop modules (atten_mean / atten_scale, cc_*_transforms, lrp_transforms) are
    # never updated, their .grad only grows, and :198 clips over ALL net.parameters(), growing norms
    # included.  Default here: those modules take no weight gradient at all (requires_grad off: no
    # wgrad launches, no AccumulateGrad additions -- ~300 per step) and the clip runs over the
    # optimised parameters; --ref-clip keeps the reference's accumulate-and-clip-over-everything.
    if not args.ref_clip:
        opt_ids = {id(p) for p in params}
        for p in net.parameters():
            if id(p) not in opt_ids:
                p.requires_grad_(False)
    if args.graph and args.precision == "fp16":
        raise SystemExit("--graph: bf16 / fp32 (fp16's GradScaler syncs the host every step)")
    # capturable Adam keeps lr and the step count on the device (graph replays update them); fused:
    # one multi-tensor kernel per step -- the foreach path with a device lr falls back to one
    # broadcast division per parameter (~1000 launches per step, rocprofv3 trace r04v)
    opt = torch.optim.Adam(params, lr=torch.tensor(args.lr, device=dev) if args.graph else args.lr,
                           capturable=args.graph, fused=os.environ.get("LIC_FUSED_ADAM", "1") != "0")
    sch = torch.optim.lr_scheduler.MultiStepLR(opt, [1500, 2500, 3500, 4000], 0.5)
    sync = D.GradAllReduce(params, world)
    # one GPU: the backward's split-K wgrad reduces as one launch after it (autograd.WgradDefer; at
    # world > 1 the eager GradAllReduce hooks read .grad during the backward).  LIC_WGRAD_DEFER=0: off
    # (--ref-clip: the accumulating gradients would be added before their reduce ran)
    wdefer = AG.WgradDefer() if (world == 1 and not args.ref_clip and
                                 os.environ.get("LIC_WGRAD_DEFER", "1") != "0") else None
    clip_params = list(net.parameters()) if args.ref_clip else params

    def backward(t):
        with wdefer if wdefer is not None else contextlib.nullcontext():
            t.backward()
    scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 10, enabled=args.precision == "fp16")
    batches = Crops(synthetic_bank(16, 2 * args.crop, 5000 + 97 * rank, dev), B, args.crop, 1234 + rank)

    grad_params = None

    def step_body(x, seed_dev=None):
        bpp, mse = net(x, "train", seed_dev=seed_dev)
        loss = args.lmbda * 255 ** 2 * mse + bpp                       # :180
        backward(loss)
        sync.finish()                                                  # RCCL all-reduce, captured too
        torch.nn.utils.clip_grad_norm_(grad_params, 1.0)               # :198
        opt.step()
        return loss.detach(), bpp.detach(), mse.detach()

    if args.graph:
        # W eager warm-up steps (Adam state, caches) on a side stream, then one capture
        static_x = batches().clone()
        seed_t = torch.zeros((1,), dtype=torch.int64, device=dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream())
        # every weight pack of the step in one launch at its start (functional.PackPlan): the last
        # warm-up step (caches already warm) records them, the captured step replays them
        plan = Fn.PackPlan() if os.environ.get("LIC_PACK_PLAN", "1") != "0" else None
        nwarm = max(2 if plan is not None else 1, args.warmup)
        with torch.cuda.stream(side):
            for k in range(nwarm):
                opt.zero_grad(set_to_none=True)
                with plan.record() if (plan is not None and k == nwarm - 1) else contextlib.nullcontext():
                    bpp, mse = net(static_x, "train", seed_dev=seed_t)
                    backward(args.lmbda * 255 ** 2 * mse + bpp)
                sync.finish()              # first collectives eagerly: communicator set up before capture
                grad_params = [p for p in clip_params if p.grad is not None]
                torch.nn.utils.clip_grad_norm_(grad_params, 1.0)
                opt.step()
                seed_t.add_(1)
        torch.cuda.current_stream().wait_stream(side)
        opt.zero_grad(set_to_none=True)
        if plan is not None:
            plan.finalize()
        torch.cuda.synchronize(dev)   # the warm-up's collectives complete before the capture starts
        sync.defer = True             # buckets launched from finish() on the capturing thread
        graph = torch.cuda.CUDAGraph()
        # the warm-up's stream: AccumulateGrad nodes stay on it.  thread_local: RCCL's watchdog thread
        # keeps querying its events during the capture (a global-mode capture makes that an error)
        with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
            if plan is not None:
                plan.launch_all()
            with plan.replay() if plan is not None else contextlib.nullcontext():
                outs = step_body(static_x, seed_t)
            seed_t.add_(1)
        if wdefer is not None:
            wdefer.finalize()

        def step():
            static_x.copy_(batches())
            graph.replay()
            return outs
    else:
        def step():
            return eager_step()

    def eager_step():
        x = batches()
        opt.zero_grad(set_to_none=True)
        bpp, mse = net(x, "train")
        loss = args.lmbda * 255 ** 2 * mse + bpp                       # :180
        backward(scaler.scale(loss))
        sync.finish()
        scaler.unscale_(opt)
        torch.nn.utils.clip_grad_norm_([p for p in clip_params if p.grad is not None], 1.0)   # :198
        scaler.step(opt)
        scaler.update()
        return loss.detach(), bpp.detach(), mse.detach()

    if args.bench:
        first = None
        for _ in range(max(1, args.warmup)):
            out = step()
            first = first if first is not None else float(out[0])
        D.barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        D.barrier(world)
        dt = D.max_over_ranks(dt, world, dev)
        last = float(out[0])
        if rank == 0:
            print(json.dumps({
                "metric": f"train images/sec ({args.crop}x{args.crop} crops, {args.arch}, batch {B}/GPU)",
                "value": round(world * B * args.steps / dt, 2), "unit": "images/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": {"fp16": "f16", "bf16": "bf16"}.get(args.precision, "f32"),
                "data": "synthetic (seeded smooth images, random crops in HBM; no DIV2K)",
                "config": {"workload": f"{args.arch} Net.forward(x,'train') + backward + grad all-reduce + clip + Adam",
                           "global_batch": world * B, "crop": args.crop, "lambda": args.lmbda,
                           "parallelism": f"data-parallel x{world} (bucketed RCCL all-reduce)",
                           "execution": "hipGraph replay of the whole step" if args.graph else "eager"},
                "loss_first_last": [round(first, 4), round(last, 4)]}), flush=True)
        D.finish(world)
        return

    for epoch in range(args.epochs):
        sums = [0.0, 0.0, 0.0]
        acc = None
        for i in range(args.steps_per_epoch):
            out = torch.stack(step())
            acc = out if acc is None else acc + out
            if (i + 1) % args.log_every == 0 or i + 1 == args.steps_per_epoch:
                vals = acc.tolist()                                      # one sync per log window
                if math.isnan(vals[0]):
                    raise Exception("NaN in loss")                      # :189-190
                sums = [s + v for s, v in zip(sums, vals)]
                acc = None
        sch.step()
        cnt = args.steps_per_epoch
        if rank == 0:
            msg = "[Epoch %04d TRAIN] Loss: %.4f bpp: %.4f mse: %.4f  " % (epoch, sums[0] / cnt, sums[1] / cnt,
                                                                          sums[2] / cnt)
            print(msg, flush=True)
            if args.checkpoint_dir:
                os.makedirs(args.checkpoint_dir, exist_ok=True)
                with open(os.path.join(args.checkpoint_dir, "train_log.txt"), "a") as fd:
                    fd.write(msg + "\n")
                if epoch % 100 == 99:
                    torch.save(net.state_dict(), "%s/%04d.ckpt" % (args.checkpoint_dir, epoch))
    D.finish(world)


if __name__ == "__main__":
    main()
