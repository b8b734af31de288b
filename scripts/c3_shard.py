"""BASELINE config 3 (10M x 1M @2e-4) with item-sharded bitmaps (DistMiner mode "shard") or
transaction-DP (--mode tx): one JSON line from rank 0.  Under torchrun the ranks use RCCL, or
gloo with KMLS_BENCH_DIST=gloo (ranks sharing one GPU)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="shard", choices=["shard", "tx"])
    ap.add_argument("--min-support", type=float, default=None)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch-div", default="", help="comma list: item_shard.BATCH_DIV sweep")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.bench import bench_mine as bm
    from kubernetes_machine_learning_server_amd.ops import native
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if os.environ.get("KMLS_BENCH_DIST") == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    N = native.require_gpu()
    ms = args.min_support if args.min_support is not None else bm.C3_MIN_SUPPORT
    from kubernetes_machine_learning_server_amd.parallel import item_shard
    for div in [int(x) for x in args.batch_div.split(",") if x] or [item_shard.BATCH_DIV]:
        item_shard.BATCH_DIV = div
        out = bm.run_config3(N, world, rank, dev, steps=args.steps, warmup=args.warmup,
                             comm="host", min_support=ms, mode=args.mode)
        if rank == 0:
            out["batch_div"] = div
            print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
