"""resource.Quantity: parse / compare / canonical format.

Behavioural parity with apimachinery's Quantity
(reference: staging/src/k8s.io/apimachinery/pkg/api/resource/quantity.go:98 parse
grammar, :276 ParseQuantity, suffix tables in suffix.go).

Internally a quantity is an exact ``fractions.Fraction`` plus the format family it was
written in (DecimalSI, BinarySI, DecimalExponent), so "288Gi" round-trips and
``Quantity("500m").milli_value() == 500`` without float error.
"""
from __future__ import annotations

import math
import re
from fractions import Fraction
from functools import lru_cache, total_ordering

DECIMAL_SI = "DecimalSI"
BINARY_SI = "BinarySI"
DECIMAL_EXPONENT = "DecimalExponent"

_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": Fraction(1),
        "k": Fraction(10 ** 3), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9), "T": Fraction(10 ** 12),
        "P": Fraction(10 ** 15), "E": Fraction(10 ** 18)}
_DEC_ORDER = [("E", 18), ("P", 15), ("T", 12), ("G", 9), ("M", 6), ("k", 3), ("", 0), ("m", -3), ("u", -6), ("n", -9)]
_BIN_ORDER = [("Ei", 60), ("Pi", 50), ("Ti", 40), ("Gi", 30), ("Mi", 20), ("Ki", 10)]

_RE = re.compile(r"^([+-]?[0-9]*\.?[0-9]*)(Ki|Mi|Gi|Ti|Pi|Ei|[numkMGTPE]|[eE][+-]?[0-9]+)?$")


class QuantityError(ValueError):
    pass


@total_ordering
class Quantity:
    __slots__ = ("value_", "format")

    def __init__(self, v="0", fmt: str | None = None):
        if isinstance(v, Quantity):
            self.value_, self.format = v.value_, v.format
            return
        if isinstance(v, (int, Fraction)):
            self.value_ = Fraction(v)
            self.format = fmt or DECIMAL_SI
            return
        if isinstance(v, float):
            self.value_ = Fraction(v).limit_denominator(10 ** 9)
            self.format = fmt or DECIMAL_SI
            return
        self.value_, self.format = _parse(str(v))
        if fmt:
            self.format = fmt

    # ------------------------------------------------------------------ values
    def value(self) -> int:
        """Integer value rounded up (Quantity.Value semantics)."""
        return math.ceil(self.value_)

    def milli_value(self) -> int:
        return math.ceil(self.value_ * 1000)

    def as_fraction(self) -> Fraction:
        return self.value_

    def is_zero(self) -> bool:
        return self.value_ == 0

    # ------------------------------------------------------------- arithmetic
    def __add__(self, o):
        # Quantity.Add: a zero receiver takes the other operand's format
        o = Quantity(o)
        return Quantity(self.value_ + o.value_, o.format if self.value_ == 0 else self.format)

    def __sub__(self, o):
        o = Quantity(o)
        return Quantity(self.value_ - o.value_, o.format if self.value_ == 0 else self.format)

    def __neg__(self):
        return Quantity(-self.value_, self.format)

    def __eq__(self, o):
        try:
            return self.value_ == Quantity(o).value_
        except (QuantityError, TypeError):
            return NotImplemented

    def __lt__(self, o):
        return self.value_ < Quantity(o).value_

    def __hash__(self):
        return hash(self.value_)

    # -------------------------------------------------------------- formatting
    def __str__(self):
        return format_quantity(self.value_, self.format)

    def __repr__(self):
        return f"Quantity({str(self)!r})"

    def to_json(self) -> str:
        return str(self)


@lru_cache(maxsize=8192)
def _parse(s: str):
    s = s.strip()
    if not s:
        raise QuantityError("quantities must match the regular expression '^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$'")
    m = _RE.match(s)
    if not m or m.group(1) in ("", "+", "-", ".", "+.", "-."):
        raise QuantityError(f"unable to parse quantity's suffix: {s!r}")
    num, suf = m.group(1), m.group(2) or ""
    try:
        base = Fraction(num)
    except ValueError as e:  # pragma: no cover - regex already guards
        raise QuantityError(str(e))
    if suf in _BIN:
        return base * _BIN[suf], BINARY_SI
    if suf[:1] in ("e", "E"):
        return base * (Fraction(10) ** int(suf[1:])), DECIMAL_EXPONENT
    return base * _DEC[suf], DECIMAL_SI


def format_quantity(v: Fraction, fmt: str) -> str:
    """Canonical form: the largest suffix that keeps an integer mantissa.

    Like apimachinery, binary format falls back to decimal for values that are not
    integral multiples of 1Ki, and sub-milli precision is rounded up to 1n granularity.
    """
    if v == 0:
        return "0"
    sign = "-" if v < 0 else ""
    a = -v if v < 0 else v
    if fmt == BINARY_SI and a.denominator == 1 and a >= 1024:
        n = a.numerator
        for suf, p in _BIN_ORDER:
            if n % (1 << p) == 0:
                return f"{sign}{n >> p}{suf}"
        return f"{sign}{n}"
    # decimal: express as integer * 10^e with e multiple of 3, e >= -9
    scaled = math.ceil(a * 10 ** 9)  # nano units, rounded up like Quantity does
    exp = -9
    while scaled % 1000 == 0 and exp < 18:
        scaled //= 1000
        exp += 3
    if fmt == DECIMAL_EXPONENT:
        return f"{sign}{scaled}" + (f"e{exp}" if exp else "")
    suf = {e: s for s, e in _DEC_ORDER}[exp]
    return f"{sign}{scaled}{suf}"


def parse_quantity(s) -> Quantity:
    return Quantity(s)


def q_value(v) -> int:
    return Quantity(v).value()


def q_milli(v) -> int:
    return Quantity(v).milli_value()
