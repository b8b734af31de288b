"""Debug: resident path with max_len=2 (with/without the device rule map)."""
import faulthandler
import numpy as np
from kubernetes_machine_learning_server_amd.data.synthetic import generate
from kubernetes_machine_learning_server_amd.ops import native
from kubernetes_machine_learning_server_amd.serve.index import name_tie_rank
faulthandler.enable()
N = native.require_gpu()
tx = generate("ds1", seed=2)
for ri in (False, True):
    g = N.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    if ri:
        g.set_tie_rank(name_tie_rank(tx.names))
    for rep in range(2):
        r = g.mine(0.01, 2, rule_index=ri)
        for k in ("parent", "item", "count", "depth"):
            a = r[k]
            print(rep, k, a.dtype, a.shape, a.flags["C_CONTIGUOUS"], int(np.asarray(a).min()), int(np.asarray(a).max()), flush=True)
        print(" stats", r["stats"], flush=True)
        print(" gpu", N.trie_digest(r["parent"], r["item"], r["count"], r["depth"])["digest"], flush=True)
