"""Host logic of the operator mirror (skyline/operators.py) that needs no device: the trigger
payload parsing must be the reference's -- String.split(",") and Long.parseLong without trim
(FlinkSkyline.java:303-305, :333-334, :627-629) -- so a payload the Java job rejects is rejected
here too (the Java drop-in, java/org/main/HipSkylineOperators.java, parses the same way)."""
import pytest

from skyline.operators import SkylineLocalProcessor, java_parse_long, java_split


@pytest.mark.parametrize("s,v", [("1000", 1000), ("+7", 7), ("-12", -12), ("0", 0),
                                 ("9223372036854775807", (1 << 63) - 1), ("-9223372036854775808", -(1 << 63))])
def test_parse_long_accepts(s, v):
    assert java_parse_long(s) == v


@pytest.mark.parametrize("s", [" 1000", "1000 ", "1_000", "", "+", "-", "1e3", "10.0", "٣", "9223372036854775808",
                               "-9223372036854775809", "0x10", "\t5"])
def test_parse_long_rejects(s):
    with pytest.raises(ValueError):
        java_parse_long(s)


@pytest.mark.parametrize("s,parts", [("q,1000", ["q", "1000"]), ("q", ["q"]), ("q,", ["q"]), ("q,,", ["q"]),
                                     (",", []), ("", [""]), (",5", ["", "5"]), ("a,b,c", ["a", "b", "c"])])
def test_split_is_javas(s, parts):
    assert java_split(s) == parts


def test_required_count_is_parsed_like_the_reference():
    assert SkylineLocalProcessor._required((0, "q1,5000", 0)) == 5000
    assert SkylineLocalProcessor._required((0, "q1", 0)) == 0          # no comma: requiredCount 0 (:305)
    assert SkylineLocalProcessor._required((0, "q1,", 0)) == 0         # "q1,".split(",") has one part
    with pytest.raises(ValueError):                                     # Long.parseLong(" 5000") throws
        SkylineLocalProcessor._required((0, "q1, 5000", 0))
