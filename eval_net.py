#!/usr/bin/env python3
"""eval_net.py — the reference CLI (eval_net.py:202-255) on the HIP path.

Same flags and per-image / summary print format as the reference (eval_net.py:105-116).
Differences: images are timed with device synchronisation (the reference's timer is
unsynchronised, :93-100); no PNG side effects; ``--all-images`` evaluates every image
(the reference only evaluates ``sorted(glob)[22:23]``, :31); ``--arch`` / ``--precision``
select the model file and the activation dtype; a missing checkpoint falls back to the
reference's seeded initialisation with a warning (no checkpoints ship with the reference).
``--pre_processing`` runs the online encoder finetune (eval_net.py:118-199) on the liblic training
path (Net.forward(x, 'train') + backward) before evaluating each image.

BASELINE config 4 (Kodak-24 R-D sweep, image-sharded over 1/2/4/8 GPUs):
``--synthetic-kodak`` stands in for the Kodak PNGs (none ship with the reference and
there is no network): 24 seeded smooth images with Kodak's shapes (18 landscape
768x512, 6 portrait 512x768 at Kodak's portrait indices).  ``--lambdas`` sweeps the
reference's lambda list; with no checkpoints each lambda's weights are the seeded
reference initialisation with seed = lambda index, or
``--weight_path`` may contain ``{lmbda}``.  ``--graph`` replays one captured hipGraph
per (lambda, image shape).  Rank 0 prints one JSON summary line (images/s of the sweep,
whole job, elapsed = MAX over ranks).
"""
import argparse
import glob
import json
import math
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def load_image(path):
    from PIL import Image
    img = Image.open(path).convert("RGB")
    data = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1).contiguous()
    return data


def pad64(data):
    """eval_net.py:68-81: pad H, W up to a multiple of 64 with the value 1.0."""
    _, h, w = data.shape
    hp = h if h % 64 == 0 else (h // 64) * 64 + 64
    wp = w if w % 64 == 0 else (w // 64) * 64 + 64
    data = torch.cat((data, torch.ones(3, hp - h, w)), 1)
    data = torch.cat((data, torch.ones(3, hp, wp - w)), 2)
    return data, h, w


KODAK_PORTRAIT = (3, 8, 9, 16, 17, 18)   # 0-based indices of Kodak's 512x768 (portrait) images
RD_LAMBDAS = (0.0018, 0.0035, 0.0067, 0.0130, 0.0250, 0.0483, 0.0932)


def synthetic_image(idx, h, w):
    """Seeded smooth stand-in for a natural image: a sum of random low-frequency
    sinusoids per channel plus mild noise, in [0, 1]."""
    g = torch.Generator().manual_seed(1000 + idx)
    yy = torch.linspace(0, 1, h).view(h, 1)
    xx = torch.linspace(0, 1, w).view(1, w)
    img = torch.zeros(3, h, w)
    for c in range(3):
        for _ in range(6):
            fy, fx = (torch.rand(2, generator=g) * 8).tolist()
            ph, amp = (torch.rand(2, generator=g) * torch.tensor([2 * math.pi, 0.25])).tolist()
            img[c] += amp * torch.sin(2 * math.pi * (fy * yy + fx * xx) + ph)
    img = 0.5 + img + 0.03 * torch.randn(3, h, w, generator=g)
    return img.clamp(0, 1)


def synthetic_kodak():
    """24 (name, [3,H,W] in [0,1]) pairs with Kodak-24's shapes."""
    return [(f"synthetic_kodim{i + 1:02d}", synthetic_image(i, *((768, 512) if i in KODAK_PORTRAIT else (512, 768))))
            for i in range(24)]


def rd_sweep(lambdas, weight_path, arch="net_ga", precision="fp32x6", is_high=False, graph=True, reps=1,
             device="cuda", batched=True):
    """BASELINE config 4: every lambda x every synthetic Kodak image, images sharded
    round-robin over ranks.  Returns (per-lambda summaries, images/s) on rank 0.

    batched (default): per lambda, each rank's images of one shape (Kodak: 18 landscape 768x512, 6
    portrait 512x768) run as ONE batch -- one net and one captured hipGraph per (lambda, shape); the
    summaries are the same per-image means (bpp of a batch of equal-sized images is the mean of their
    bpps; PSNR is the mean of per-image PSNRs, net_ga.py:1141-1142).  batched=False: one image per
    forward (the reference's loop).  Default precision: fp32x6, the bench's gated fp32-grade path."""
    from lic_amd.model import net_ga, net_unet_ha_hs
    from lic_amd import distributed as D
    mod = net_ga if arch == "net_ga" else net_unet_ha_hs
    rank, world, local = D.init("nccl")
    if world > 1 or torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    mine = D.shard(synthetic_kodak(), rank, world)
    # shape -> padded [B, 3, H, W] batch in [-1, 1], in first-seen order
    groups = []
    for name, img in mine:
        data, h, w = pad64(img)
        x = data.unsqueeze(0) * 2.0 - 1.0
        for grp in groups:
            if grp[0] == (h, w):
                grp[1].append(x)
                break
        else:
            groups.append(((h, w), [x]))
    batches = [(hw, torch.cat(xs, 0).to(device)) for hw, xs in groups]
    summaries, total_time = [], 0.0
    for li, lmbda in enumerate(lambdas):
        sums = [0.0, 0.0, 0.0, 0.0]  # bpp, psnr, mse, rd (sums over images)
        for (h, w), X in batches:
            B = X.shape[0] if batched else 1
            torch.manual_seed(li)
            net = mod.Net((B, h, w, 3), (B, h, w, 3), is_high, False, precision=precision).to(device)
            wp = weight_path.format(lmbda=lmbda) if weight_path else ""
            if wp and os.path.exists(wp):
                net.load_state_dict(torch.load(wp, map_location="cpu", weights_only=True), strict=True)
            else:
                net_ga.synthetic_syntax_bias_(net, li)
            xin = X[:B].clone()
            g = out = None
            if graph:
                net(xin, 'test')
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    net(xin, 'test')
                torch.cuda.current_stream().wait_stream(s)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    out = net(xin, 'test')
            for i0 in range(0, X.shape[0], B):
                xin.copy_(X[i0:i0 + B])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    if graph:
                        g.replay()
                        bpp, v_mse, v_psnr = out
                    else:
                        bpp, v_mse, v_psnr = net(xin, 'test')
                torch.cuda.synchronize()
                total_time += (time.perf_counter() - t0) / reps
                b, p, msum = bpp.item(), v_psnr.item(), v_mse.double().sum().item()
                sums[0] += B * b; sums[1] += B * p; sums[2] += msum; sums[3] += B * b + lmbda * msum
            # the graph before the net whose buffers it replays; memory back before the next shape
            del g, out, net, xin
            torch.cuda.synchronize()
        sums = D.sum_over_ranks(sums + [len(mine)], world, device)
        cnt = sums[4]
        summaries.append({"lambda": lmbda, "bpp": sums[0] / cnt, "psnr": sums[1] / cnt, "mse": sums[2] / cnt,
                          "rd": sums[3] / cnt, "images": int(cnt)})
        if rank == 0:
            print('[lambda %.4f] bpp: %.4f psnr: %.4f v_mse: %.4f bpp+lambda*mse: %.4f' % (
                lmbda, sums[0] / cnt, sums[1] / cnt, sums[2] / cnt, sums[3] / cnt), flush=True)
    # elapsed = slowest rank's forward time; images = all ranks' images over the sweep
    elapsed = D.max_over_ranks(total_time, world, device)
    n_img = len(lambdas) * 24
    torch.cuda.synchronize()
    D.finish(world)
    return summaries, n_img / elapsed, world


def finetune_encoder(net, data, lmbda, tune_iter):
    """Online encoder finetune (eval_net.py:160-179): Adam(a_model, 1e-5), MultiStepLR([50], 0.5),
    loss = lambda * mse + bpp in train mode, post-processing off during the finetune."""
    opt_enc = torch.optim.Adam(net.a_model.parameters(), lr=1e-5)
    sch = torch.optim.lr_scheduler.MultiStepLR(opt_enc, [50], 0.5)
    post = net.post_processing
    net.post_processing = False
    for _ in range(tune_iter):
        train_bpp, train_mse = net(data, 'train')
        train_loss = (lmbda * train_mse + train_bpp).mean()
        opt_enc.zero_grad()
        train_loss.backward()
        opt_enc.step()
        sch.step()
    net.post_processing = post


def val(data_path, weight_path, lmbda, is_high, post_processing, pre_processing, tune_iter, arch="net_ga",
        precision="fp32", all_images=False, device="cuda", noise_seed=None):
    from lic_amd.model import net_ga, net_unet_ha_hs
    from lic_amd import distributed as D
    mod = net_ga if arch == "net_ga" else net_unet_ha_hs
    # one process per GPU under torch.distributed.run: images round-robin over ranks,
    # one all-reduce of the summary sums at the end
    rank, world, local = D.init("nccl")
    if world > 1:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    images = list(sorted(glob.glob(data_path)))
    if not all_images:
        images = images[22:23]
    images = D.shard(images, rank, world)
    list_eval_bpp = list_v_psnr = list_v_mse = 0.0
    cnt = 0
    sum_time = 0.0
    for img_name in images:
        print("img_name:", img_name)
        data, h, w = pad64(load_image(img_name))
        data = (data.unsqueeze(0) * 2.0 - 1.0).to(device)
        torch.manual_seed(0)
        net = mod.Net((1, h, w, 3), (1, h, w, 3), is_high, post_processing, precision=precision).to(device)
        if weight_path and os.path.exists(weight_path):
            net.load_state_dict(torch.load(weight_path, map_location="cpu", weights_only=True), strict=True)
        else:
            print(f"warning: checkpoint {weight_path!r} not found; using the seeded reference initialisation")
            net_ga.synthetic_syntax_bias_(net)
        torch.cuda.synchronize()
        begin_time = time.time()
        if pre_processing:
            finetune_encoder(net, data, lmbda, tune_iter)
        with torch.no_grad():
            eval_bpp, v_mse, v_psnr = net(data, 'test', noise_seed=None if noise_seed is None else noise_seed + cnt)
        torch.cuda.synchronize()
        end_time = time.time()
        sum_time += end_time - begin_time
        list_eval_bpp += eval_bpp.mean().item()
        list_v_psnr += v_psnr.mean().item()
        list_v_mse += v_mse.mean().item()
        print(end_time - begin_time, img_name, eval_bpp.mean().item(), v_psnr.mean().item(),
              (eval_bpp + lmbda * v_mse).cpu().item())
        cnt += 1
    sum_time, list_eval_bpp, list_v_psnr, list_v_mse, cnt = D.sum_over_ranks(
        [sum_time, list_eval_bpp, list_v_psnr, list_v_mse, cnt], world, device)
    if cnt and rank == 0 and pre_processing:
        print('[WITH PRE-PROCESSING] bpp: %.4f psnr: %.4f' % (list_eval_bpp / cnt, list_v_psnr / cnt))
    elif cnt and rank == 0:
        print('[WITHOUT PRE-PROCESSING] ave_time:%.4f bpp: %.4f psnr: %.4f  v_mse: %.4f' % (
            sum_time / cnt, list_eval_bpp / cnt, list_v_psnr / cnt, list_v_mse / cnt))
    D.finish(world)


def main(argv=None):
    parser = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    parser.add_argument("--data_path", default="/media/yang/Pytorch/buxiaobu/code/My_dataset/kodak/*",
                        help="Directory of Testset Images")
    parser.add_argument("--weight_path", default="", help="Path of Checkpoint")
    parser.add_argument("--high", action="store_true", help="Using High Bitrate Model")
    parser.add_argument("--post_processing", action="store_true", help="Using Post Processing")
    parser.add_argument("--pre_processing", action="store_true", help="Using Pre Processing (Online Finetuning)")
    parser.add_argument("--lambda", type=float, default=0.0067, dest="lmbda", help="Lambda for rate-distortion tradeoff.")
    parser.add_argument("--tune_iter", type=int, default=100, help="Finetune Iteration")
    parser.add_argument("--arch", default="net_ga", choices=["net_ga", "net_unet_ha_hs"])
    parser.add_argument("--precision", default="fp32", choices=["fp32", "fp32x6", "fp32x3", "bf16", "fp16"],
                        help="fp32: exact fp32 (the reference's arithmetic); fp32x6: fp32 activations and "
                             "accumulation, products from six bf16 MFMA products of exact three-part splits "
                             "(fp32 grade, faster); fp32x3: fp16-part products (~22 bits, not fp32 grade); "
                             "bf16 / fp16: 16-bit activations (not parity grade)")
    parser.add_argument("--all-images", action="store_true", dest="all_images")
    parser.add_argument("--noise_seed", type=int, default=None,
                        help="price y + U(-1/2,1/2) as the reference's eval does (its nets are never put in "
                             "eval mode); seeded, image k uses seed + k.  Default: dequantize semantics")
    parser.add_argument("--synthetic-kodak", action="store_true", dest="synthetic_kodak",
                        help="BASELINE config 4: R-D sweep over 24 synthetic Kodak-shaped images")
    parser.add_argument("--lambdas", default=",".join(str(v) for v in RD_LAMBDAS),
                        help="comma-separated lambda list for --synthetic-kodak")
    parser.add_argument("--graph", action="store_true", help="hipGraph replay per (lambda, shape)")
    parser.add_argument("--per-image", action="store_true", dest="per_image",
                        help="--synthetic-kodak: one image per forward instead of one batch per image shape")
    parser.add_argument("--gpus", type=int, default=1,
                        help="ranks (one per GPU); without torchrun this process starts them itself")
    args = parser.parse_args(argv)
    # the sweep defaults to the bench's fp32-grade fp32x6; the single-image CLI keeps exact fp32
    args.precision_given = any(a == "--precision" or a.startswith("--precision=")
                               for a in (sys.argv[1:] if argv is None else argv))
    from lic_amd import distributed as D
    if args.gpus > 1 and not D.launched():
        # one process per GPU, started before this process touches the GPU (no re-exec)
        sys.exit(D.launch_workers([sys.executable, os.path.abspath(__file__)] + (sys.argv[1:] if argv is None
                                                                                 else list(argv)), args.gpus))
    if D.launched() and D.env_rank()[1] != args.gpus and args.gpus > 1:
        raise SystemExit(f"eval_net.py: --gpus {args.gpus} but the launcher started {D.env_rank()[1]} ranks")
    if args.synthetic_kodak:
        lambdas = [float(v) for v in args.lambdas.split(",") if v]
        prec = args.precision if args.precision_given else "fp32x6"
        summ, ips, world = rd_sweep(lambdas, args.weight_path, arch=args.arch, precision=prec,
                                    is_high=args.high, graph=args.graph, batched=not args.per_image)
        if int(os.environ.get("RANK", 0)) == 0:
            print(json.dumps({"metric": "images/sec encode+decode (Kodak-24 R-D sweep, 768x512)",
                              "value": round(ips, 2), "unit": "images/s", "n_gpus": world,
                              "arch": args.arch, "precision": prec, "graph": args.graph,
                              "batching": "per image" if args.per_image else "one batch per (lambda, image shape)",
                              "data": "synthetic Kodak-shaped images, seeded weights per lambda",
                              "rd": summ}), flush=True)
        return
    print(args.weight_path)
    val(args.data_path, args.weight_path, args.lmbda, args.high, args.post_processing, args.pre_processing,
        args.tune_iter, arch=args.arch, precision=args.precision, all_images=args.all_images,
        noise_seed=args.noise_seed)


if __name__ == "__main__":
    main()
