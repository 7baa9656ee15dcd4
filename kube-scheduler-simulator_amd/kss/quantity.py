"""Exact Kubernetes resource.Quantity parsing (k8s.io/apimachinery/pkg/api/resource).

Only what the scheduler path reads is restated: parse a quantity string into an
exact rational and expose ``Value()`` / ``MilliValue()`` with the upstream
rounding (ScaledValue rounds away from zero, i.e. up for the non-negative
quantities resource requests carry).
"""
from __future__ import annotations

from fractions import Fraction
import math
import re

_BINARY = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}
_DECIMAL = {"n": Fraction(1, 10**9), "u": Fraction(1, 10**6), "m": Fraction(1, 1000), "": Fraction(1),
            "k": Fraction(10**3), "M": Fraction(10**6), "G": Fraction(10**9), "T": Fraction(10**12),
            "P": Fraction(10**15), "E": Fraction(10**18)}
_NUM = re.compile(r"^([+-]?)(\d*)(?:\.(\d*))?(.*)$")


class QuantityError(ValueError):
    pass


def parse(q) -> Fraction:
    """Parse ``q`` (str, int or float) into an exact Fraction."""
    if isinstance(q, bool):
        raise QuantityError(f"bad quantity {q!r}")
    if isinstance(q, int):
        return Fraction(q)
    if isinstance(q, float):
        return Fraction(str(q))
    s = str(q).strip()
    m = _NUM.match(s)
    if not m or (m.group(2) == "" and not m.group(3)):
        raise QuantityError(f"bad quantity {q!r}")
    sign, ip, fp, suf = m.group(1), m.group(2) or "0", m.group(3) or "", m.group(4)
    mant = Fraction(int(ip + fp) if (ip + fp) else 0, 10 ** len(fp))
    if sign == "-":
        mant = -mant
    if suf in _BINARY:
        return mant * _BINARY[suf]
    if suf in _DECIMAL:
        return mant * _DECIMAL[suf]
    if suf[:1] in ("e", "E"):
        try:
            e = int(suf[1:])
        except ValueError as exc:
            raise QuantityError(f"bad quantity {q!r}") from exc
        return mant * (Fraction(10) ** e)
    raise QuantityError(f"bad quantity suffix in {q!r}")


def _ceil_away(x: Fraction) -> int:
    return math.ceil(x) if x >= 0 else math.floor(x)


def value(q) -> int:
    """resource.Quantity.Value(): rounded away from zero to an integer."""
    return _ceil_away(parse(q))


def milli_value(q) -> int:
    """resource.Quantity.MilliValue()."""
    return _ceil_away(parse(q) * 1000)
