"""JVM semantics helpers (fastapriori_amd/utils/jvm.py)."""
from fastapriori_amd.utils.jvm import (java_parse_int, java_split_ws, java_string_key, java_trim,
                                       split_lines)


def test_split_ws():
    assert java_split_ws("") == [""]
    assert java_split_ws("   ") == [""]
    assert java_split_ws(" a\tb  c ") == ["a", "b", "c"]
    assert java_split_ws("a\x0bb\x0cc") == ["a", "b", "c"]
    assert java_split_ws("\x01a\x01") == ["a"]          # trim() strips <= U+0020
    assert java_split_ws("a\x01b") == ["a\x01b"]        # ... but \\s does not match \x01


def test_trim():
    assert java_trim("\x00\x1f x \x20") == "x"


def test_string_order_utf16():
    # U+FF61 (BMP) sorts AFTER U+1F600 (surrogates 0xD83D...) in Java, before it by code point
    a, b = "｡", "\U0001F600"
    assert java_string_key(b) < java_string_key(a)
    assert sorted(["10", "1 5", "9"], key=java_string_key) == ["1 5", "10", "9"]


def test_parse_int():
    assert java_parse_int("+7") == 7 and java_parse_int("-0") == 0 and java_parse_int("007") == 7
    assert java_parse_int("2147483648") is None and java_parse_int("1.0") is None
    assert java_parse_int("") is None


def test_split_lines():
    assert split_lines("a\nb\r\nc\rd") == ["a", "b", "c", "d"]
    assert split_lines("a\n") == ["a"]
    assert split_lines("\n\n") == ["", ""]
    assert split_lines("a\r\r\nb") == ["a", "", "b"]


def test_numeric_f1_ties_follow_java_string_order():
    # equal counts everywhere: ranks must follow Java String order of the tokens
    # (numeric keys in FastApriori._frequent_items, no strings built for the sort)
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.utils.io import parse_bytes
    toks = ["0", "1", "2", "10", "19", "100", "1000000000", "999", "2147483646", "21474836"]
    data = ("\n".join([" ".join(toks)] * 5 + [""] * 5) + "\n").encode()
    res = FastApriori(0.1, config=MinerConfig(min_support=0.1)).run(parse_bytes(data))
    assert res.items == sorted(toks + [""])
