"""Generate tests/golden/extender_known_answer.json from the reference's own files: the
second reference-held known answer, in which one node already holds a pod.

Inputs (read at generation time only, in the build container):
  /root/reference/simulator/docs/plugin-extender.md:80-109  (expected annotations of pod-8ldq5;
                                                             repeated in external-scheduler.md)
  /root/reference/web/components/lib/templates/node.yaml    (node template, both nodes)
  /root/reference/web/components/lib/templates/pod.yaml     (pod template: the pending pod and
                                                             the pod already bound to node-282x7)
The expected scores pin the bound pod: node-282x7's NodeResourcesFit 47 =
floor((floor((4000-200)*100/4000) + floor((32Gi-32Gi)*100/32Gi)) / 2) and
BalancedAllocation 52 = int64((1 - |0.05 - 1.0| / 2) * 100) are those of a node whose
Requested is one template pod (100m / 16Gi): memory fits exactly (16Gi of 16Gi free).
The out-of-tree sample plugin NodeNumber and the extender's custom
"noderesourcefit-prefilter-data" result are dropped: neither is in the default profile.
The reference is never read at test time; the JSON is the committed fixture.
"""
import json
import os

import yaml

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "extender_known_answer.json")


def main():
    node = yaml.safe_load(open(f"{REF}/web/components/lib/templates/node.yaml"))
    pod = yaml.safe_load(open(f"{REF}/web/components/lib/templates/pod.yaml"))
    md = open(f"{REF}/simulator/docs/plugin-extender.md").read()
    start = md.index("kind: Pod\napiVersion: v1\nmetadata:\n  name: pod-8ldq5")
    doc = yaml.safe_load(md[start:md.index("```", start)])
    ann = doc["metadata"]["annotations"]
    names = list(json.loads(ann["scheduler-simulator/filter-result"]).keys())
    nodes = []
    for nm in names:
        n = json.loads(json.dumps(node))
        n["metadata"].pop("generateName", None)
        n["metadata"]["name"] = nm
        nodes.append(n)
    pending = json.loads(json.dumps(pod))
    pending["metadata"].pop("generateName", None)
    pending["metadata"]["name"] = doc["metadata"]["name"]
    bound = json.loads(json.dumps(pod))
    bound["metadata"].pop("generateName", None)
    bound["metadata"]["name"] = "pod-bound-0"
    bound["spec"]["nodeName"] = "node-282x7"
    expected = {}
    for k, v in ann.items():
        if k in ("scheduler-simulator/result-history", "noderesourcefit-prefilter-data"):
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
    json.dump({"source": "simulator/docs/plugin-extender.md:80-109; web/components/lib/templates/{node,pod}.yaml",
               "nodes": nodes, "bound": [bound], "pod": pending, "expected": expected}, open(OUT, "w"), indent=1,
              sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
