import json
d = json.loads(open("gpurun_out/pp.json").read().strip().splitlines()[-1])
print({k: d[k] for k in ("eval_us", "eval_slim_us", "eval_view_us", "commit_us")})
