"""Multi-process check of DistMiner's replicated mode on ONE GPU (every rank uses cuda:0,
collectives over gloo): the global itemset count equals the single-process count and the
gathered trie equals the CPU miner's.  Launched by tests/test_gpu_kernels.py through
torch.distributed.run (127.0.0.1 rendezvous)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist


def main():
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner, gather_trie
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    tx = generate("ds2_weak", seed=8)
    dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, 0.03, device=0)
    assert dm.mode == "replicate", dm.mode
    r = dm.step(download=True)
    N = native.load()
    ref = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.03)
    merged = gather_trie(r["trie"], rank, world, int(r["stats"]["n_frequent_items"]))
    ok = int(r["stats"]["global_itemsets"]) == int(ref["stats"]["n_itemsets"])
    if rank == 0:
        ok = ok and len(merged["item"]) == len(ref["item"])
        ok = ok and np.array_equal(np.sort(merged["count"]), np.sort(ref["count"]))
        print("replicate_check", "OK" if ok else "MISMATCH", r["stats"]["global_itemsets"],
              ref["stats"]["n_itemsets"], flush=True)
    # bench.py's timed loop: launch-ahead steps without the per-step count all-reduce, then one
    # reduction of the last step's per-rank counts
    for i in range(4):
        st = dm.step(download=True, reduce_count=False, prefetch=i < 3)["stats"]
    ok = ok and dm.global_itemsets() == int(ref["stats"]["n_itemsets"])
    ok = ok and "adopted" in "".join(st.get("phases_ms", {}).keys())
    if rank == 0:
        print("replicate_check pipelined", "OK" if ok else "MISMATCH", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
