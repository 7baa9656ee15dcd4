import os, sys
sys.path.insert(0, "kube-scheduler-simulator_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
import numpy as np
import oracle_c
from kss import abi, native
from kss.synth import SEED_BASE
for cursor, opts in ((0, {}), (2321, {}), (2321, {"xcd": 0}), (2321, {"shards": 1})):
    native.reset_options()
    for k, v in opts.items(): native.set_option(k, v)
    p = abi.default_profile(); p.pct_nodes_to_score = 0
    n, N = 20, 5000 if "shards" not in opts else 1000
    s = native.Synth(3, SEED_BASE + 3, N, n)
    ch_o, res, st = oracle_c.schedule(p, s.cluster, s.pods, n, N, record="meta", threads=8, n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms, cursor=cursor)
    ctx = native.Context(p); ctx.load(s.cluster); ctx.stage(s.pods); ctx.set_next_start_node_index(cursor)
    ch = ctx.run_staged(n); meta = ctx.fetch_meta(n)
    print(cursor, opts, ctx.last_kernel(), ctx.last_geometry(), "next", ctx.next_start_node_index(), st["next_start"])
    for j in range(6): print("  ", j, ch[j], ch_o[j], "nf", meta[j,1], res.meta(j)["n_feasible"])
    ctx.close()
