"""Phase stamps of a k_simple / k_spread run (KSS_STAMPS_FILE), one line per shard count:

    python tools/c2_stamps.py CONFIG [SHARDS ...]     (SHARDS 0 = the library's own choice)

CONFIG is a BASELINE config index (2 = C2, 3 = C3, 4 = C4); 1000 pods of it are scheduled
per shard count and tools/stamps.py summarises shard 0's phases.  STAMP_OPTS="name=v,..." sets
library options first (e.g. no_spread=1: the general kernel k_schedule, the per-pod service's
chain); STAMP_PCT sets percentageOfNodesToScore (default 100; 0 = the adaptive window)."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import stamps  # noqa: E402
from kss import abi, native  # noqa: E402
from kss.synth import DEFAULT_SIZES, SEED_BASE  # noqa: E402


def main():
    cfg = int(sys.argv[1])
    n_nodes = DEFAULT_SIZES[cfg][0]
    for w in [int(x) for x in sys.argv[2:]] or [0]:
        path = os.path.join(tempfile.mkdtemp(prefix="kss_stamps_"), "stamps.bin")
        native.set_stamps_file(path)
        for kv in filter(None, os.environ.get("STAMP_OPTS", "").split(",")):
            k, v = kv.split("=")
            native.set_option(k, int(v))
        native.set_option("shards", w)
        s = native.Synth(cfg, SEED_BASE + cfg, n_nodes, 1000)
        prof = abi.default_profile()
        prof.pct_nodes_to_score = int(os.environ.get("STAMP_PCT", "100"))
        ctx = native.Context(prof, device=0)
        ctx.load(s.cluster)
        ctx.stage(s.pods)
        ctx.run_staged(s.n_pods)
        ctx.close()
        s.close()
        print(f"C{cfg} shards={w or 'auto'}: {stamps.summarise(path)}", flush=True)


if __name__ == "__main__":
    main()
