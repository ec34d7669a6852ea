"""JVM value semantics the reference inherits and that leak into its outputs.

The reference is Scala on the JVM; three JVM behaviours are observable in its
files and must be reproduced exactly:

* ``String`` ordering (``Utils.scala:39`` sorts freqItemset lines with the
  implicit ``Ordering[String]`` = ``String.compareTo``): lexicographic over
  UTF-16 code units.  Byte order of UTF-16-BE is exactly that order, and for
  pure ASCII it equals plain byte order.
* ``String.toInt`` (``AssociationRules.scala:117-119`` rule tiebreak) =
  ``Integer.parseInt``: optional sign, decimal digits, 32-bit range.
* ``String.trim`` / ``split("\\s+")`` line tokenisation (``Utils.scala:21``).
"""
from __future__ import annotations

import math
import re

INT_MIN = -(2 ** 31)
INT_MAX = 2 ** 31 - 1

# Java regex \s == [ \t\n\x0B\f\r]
_JAVA_WS = re.compile(r"[ \t\n\x0b\f\r]+")
_JAVA_INT = re.compile(r"[+-]?\d+")


def java_string_key(s: str) -> bytes:
    """Sort key reproducing ``java.lang.String.compareTo`` (UTF-16 code units)."""
    if s.isascii():
        return s.encode("ascii")
    return s.encode("utf-16-be", "surrogatepass")


def item_tiebreak_key(s: str, tiebreak: str = "string"):
    """Order of frequent items with equal counts (the rank tiebreak).
    The reference keeps Spark's post-shuffle collect() order, which is not
    reproducible outside Spark; the rank only orders the tokens inside an itemset line
    (and so the line sort), never which itemsets, counts or rules come out.
    "string": java.lang.String order (the default); "numeric": integer tokens by value
    (Integer.parseInt range), before the other tokens in String order."""
    if tiebreak == "numeric":
        v = java_parse_int(s)
        return (0, v, b"") if v is not None else (1, 0, java_string_key(s))
    return java_string_key(s)


def java_trim(s: str) -> str:
    """``String.trim``: strip every char <= U+0020 from both ends."""
    b, e = 0, len(s)
    while b < e and ord(s[b]) <= 0x20:
        b += 1
    while e > b and ord(s[e - 1]) <= 0x20:
        e -= 1
    return s[b:e]


def java_split_ws(line: str) -> list[str]:
    """``line.trim().split("\\\\s+")`` exactly as ``Utils.scala:21`` does it.

    An empty (or all-blank) line yields ``[""]`` — one empty token, which the
    reference counts like any other token.  Java's ``split`` drops trailing
    empty strings but keeps a leading one; after ``trim`` a leading empty
    string can only arise from the empty input itself.
    """
    t = java_trim(line)
    if t == "":
        return [""]
    parts = _JAVA_WS.split(t)
    while len(parts) > 1 and parts[-1] == "":
        parts.pop()
    return parts


def java_parse_int(s: str) -> int | None:
    """``Integer.parseInt`` or ``None`` where the JVM would throw."""
    if not _JAVA_INT.fullmatch(s):
        return None
    v = int(s)
    if v < INT_MIN or v > INT_MAX:
        return None
    return v


def min_count(min_support: float, n: int) -> int:
    """``math.ceil(minSupport * count).toInt`` (``FastApriori.scala:38-39``).

    IEEE double product, ceil, then Double->Int (saturating, truncating).
    """
    v = math.ceil(float(min_support) * float(n))
    return int(max(min(v, INT_MAX), INT_MIN))


def split_lines(data: str) -> list[str]:
    """Hadoop ``LineRecordReader`` line splitting: ``\\n``, ``\\r\\n`` or ``\\r``.

    A terminator at the very end of the data does not start an extra line.
    """
    out: list[str] = []
    i, n, start = 0, len(data), 0
    while i < n:
        c = data[i]
        if c == "\n" or c == "\r":
            out.append(data[start:i])
            if c == "\r" and i + 1 < n and data[i + 1] == "\n":
                i += 1
            start = i + 1
        i += 1
    if start < n:
        out.append(data[start:])
    return out


def rule_tiebreak_key(token: str):
    """Total order extending the reference's ``freqItems(cons).toInt`` tiebreak.

    The reference throws ``NumberFormatException`` when a confidence tie hits a
    non-integer token.  Documented divergence: integers
    first (by value), then non-integer tokens by Java string order; equal ints
    with different spellings ("01" vs "1") fall back to string order so the
    sort is deterministic.
    """
    v = java_parse_int(token)
    if v is None:
        return (1, 0, java_string_key(token))
    return (0, v, java_string_key(token))
