"""Generate tests/golden/readme_known_answer.json from the reference's own files.

Inputs (read at generation time only, in the build container):
  /root/reference/web/components/lib/templates/node.yaml  (node template, used twice)
  /root/reference/web/components/lib/templates/pod.yaml   (pod template)
  /root/reference/README.md:61-79                         (expected annotations)
The reference is never read at test time; the JSON is the committed fixture.
The out-of-tree sample plugin "NodeNumber" (simulator/docs/sample) is dropped from
the expected maps because it is not part of the default profile.
"""
import json
import os
import re

import yaml

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "readme_known_answer.json")


def main():
    node = yaml.safe_load(open(f"{REF}/web/components/lib/templates/node.yaml"))
    pod = yaml.safe_load(open(f"{REF}/web/components/lib/templates/pod.yaml"))
    readme = open(f"{REF}/README.md").read()
    start = readme.index("kind: Pod\nkind: Pod") if "kind: Pod\nkind: Pod" in readme else readme.index("kind: Pod")
    block = readme[start:readme.index("```", start)]
    doc = yaml.safe_load(block)
    ann = doc["metadata"]["annotations"]
    names = list(json.loads(ann["scheduler-simulator/filter-result"]).keys())
    nodes = []
    for nm in names:
        n = json.loads(json.dumps(node))
        n["metadata"].pop("generateName", None)
        n["metadata"]["name"] = nm
        nodes.append(n)
    pod = json.loads(json.dumps(pod))
    pod["metadata"].pop("generateName", None)
    pod["metadata"]["name"] = doc["metadata"]["name"]
    expected = {}
    for k, v in ann.items():
        if k == "scheduler-simulator/result-history":
            continue
        if isinstance(v, str) and v.startswith("{") and v != "{}":
            m = json.loads(v)
            for nk in list(m):
                if isinstance(m[nk], dict):
                    m[nk].pop("NodeNumber", None)
            m.pop("NodeNumber", None)
            expected[k] = m
        else:
            expected[k] = v
    json.dump({"source": "README.md:61-79; web/components/lib/templates/{node,pod}.yaml",
               "nodes": nodes, "pod": pod, "expected": expected}, open(OUT, "w"), indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
