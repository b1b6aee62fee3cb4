#!/usr/bin/env python3
"""eval_net.py — the reference CLI (eval_net.py:202-255) on the HIP path.

Same flags and per-image / summary print format as the reference (eval_net.py:105-116).
Differences: images are timed with device synchronisation (the reference's timer is
unsynchronised, :93-100); no PNG side effects; ``--all-images`` evaluates every image
(the reference only evaluates ``sorted(glob)[22:23]``, :31); ``--arch`` / ``--precision``
select the model file and the activation dtype; a missing checkpoint falls back to the
reference's seeded initialisation with a warning (no checkpoints ship with the reference).
``--pre_processing`` (online finetune) needs the training path and is not available yet.
"""
import argparse
import glob
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


def val(data_path, weight_path, lmbda, is_high, post_processing, pre_processing, tune_iter, arch="net_ga",
        precision="fp32", all_images=False, device="cuda"):
    if pre_processing:
        raise NotImplementedError("--pre_processing (online encoder finetune) needs the training path "
                                  "(SURVEY.md 8(f) rank 4)")
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
        torch.cuda.synchronize()
        begin_time = time.time()
        with torch.no_grad():
            eval_bpp, v_mse, v_psnr = net(data, 'test')
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
    if cnt and rank == 0:
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
    parser.add_argument("--precision", default="fp32", choices=["fp32", "fp16"])
    parser.add_argument("--all-images", action="store_true", dest="all_images")
    args = parser.parse_args(argv)
    print(args.weight_path)
    val(args.data_path, args.weight_path, args.lmbda, args.high, args.post_processing, args.pre_processing,
        args.tune_iter, arch=args.arch, precision=args.precision, all_images=args.all_images)


if __name__ == "__main__":
    main()
