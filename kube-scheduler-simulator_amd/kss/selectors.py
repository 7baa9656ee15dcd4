"""Label selectors over plain dict labels (k8s.io/apimachinery labels + metav1 helpers).

Host-side only: used by the compiler to decide which pod classes / term types a
selector matches, so the device only ever sees integer id lists.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple


class SelectorError(ValueError):
    pass


@dataclass(frozen=True)
class Selector:
    """kind: 'nothing' | 'everything' | 'reqs'; reqs: ((key, op, values), ...)."""

    kind: str
    reqs: Tuple[Tuple[str, str, Tuple[str, ...]], ...] = ()

    def empty(self) -> bool:
        # internalSelector.Empty(): no requirements (Everything).  nothingSelector.Empty() is false.
        return self.kind == "everything"

    def matches(self, labels: Optional[Dict[str, str]]) -> bool:
        labels = labels or {}
        if self.kind == "nothing":
            return False
        if self.kind == "everything":
            return True
        for key, op, vals in self.reqs:
            if not requirement_matches(key, op, vals, labels):
                return False
        return True

    def canonical(self) -> str:
        if self.kind != "reqs":
            return self.kind
        return "&".join(f"{k}|{op}|{','.join(v)}" for k, op, v in sorted(self.reqs))


NOTHING = Selector("nothing")
EVERYTHING = Selector("everything")


def requirement_matches(key: str, op: str, vals, labels: Dict[str, str]) -> bool:
    """labels.Requirement.Matches (apimachinery/pkg/labels/selector.go)."""
    has = key in labels
    if op in ("In", "=", "=="):
        return has and labels[key] in vals
    if op in ("NotIn", "!="):
        return (not has) or labels[key] not in vals
    if op == "Exists":
        return has
    if op == "DoesNotExist":
        return not has
    if op in ("Gt", "Lt"):
        if not has:
            return False
        lv = parse_int(labels[key])
        if lv is None or len(vals) != 1:
            return False
        rv = parse_int(vals[0])
        if rv is None:
            return False
        return lv > rv if op == "Gt" else lv < rv
    return False


def parse_int(s: str) -> Optional[int]:
    """strconv.ParseInt(s, 10, 64)."""
    if not isinstance(s, str) or s == "":
        return None
    body = s[1:] if s[0] in "+-" else s
    if body == "" or not body.isdigit() or not body.isascii():
        return None
    v = int(s)
    if v < -(2**63) or v > 2**63 - 1:
        return None
    return v


def label_selector_as_selector(ls) -> Selector:
    """metav1.LabelSelectorAsSelector: nil -> Nothing, {} -> Everything."""
    if ls is None:
        return NOTHING
    ml = ls.get("matchLabels") or {}
    me = ls.get("matchExpressions") or []
    if len(ml) + len(me) == 0:
        return EVERYTHING
    reqs: List[Tuple[str, str, Tuple[str, ...]]] = []
    for k, v in ml.items():
        reqs.append((k, "=", (v,)))
    for e in me:
        op = e.get("operator")
        vals = tuple(e.get("values") or ())
        if op not in ("In", "NotIn", "Exists", "DoesNotExist"):
            raise SelectorError(f"{op!r} is not a valid label selector operator")
        if op in ("In", "NotIn") and len(vals) == 0:
            raise SelectorError("for 'in', 'notin' operators, values set can't be empty")
        if op in ("Exists", "DoesNotExist") and len(vals) != 0:
            raise SelectorError("values set must be empty for exists and does not exist")
        reqs.append((e["key"], op, vals))
    return Selector("reqs", tuple(reqs))


def selector_from_set(m: Dict[str, str]) -> Selector:
    """labels.SelectorFromSet: empty set -> Everything."""
    if not m:
        return EVERYTHING
    return Selector("reqs", tuple((k, "=", (v,)) for k, v in m.items()))
