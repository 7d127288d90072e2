"""Pin the record-assembly oracle (oracle/assembly.py) to the reference's Dremel test:
TestColumnIO.expectedEventsForR1 (parquet-column/src/test/java/org/apache/parquet/io/TestColumnIO.java:114-142)
for the Document schema of org.apache.parquet.example.Paper (parquet-column/src/main/java/org/apache/parquet/example/Paper.java),
projected onto each leaf column. The column stripes (r, d, value) are those of the Dremel paper's
records r1 / r2 as parquet-mr writes them."""
import pytest

from oracle import assembly as A

R, O, P = A.REQUIRED, A.OPTIONAL, A.REPEATED

# leaf -> (names, repetitions, [(r, d, value-or-None)] for r1 then r2)
PAPER = {
    "DocId": (["DocId"], [R], [(0, 0, 10)], [(0, 0, 20)]),
    "Links.Backward": (["Links", "Backward"], [O, P], [(0, 1, None)], [(0, 2, 10), (1, 2, 30)]),
    "Links.Forward": (["Links", "Forward"], [O, P], [(0, 2, 20), (1, 2, 40), (1, 2, 60)], [(0, 2, 80)]),
    "Name.Language.Code": (["Name", "Language", "Code"], [P, P, R],
                           [(0, 2, b"en-us"), (2, 2, b"en"), (1, 1, None), (1, 2, b"en-gb")], [(0, 1, None)]),
    "Name.Language.Country": (["Name", "Language", "Country"], [P, P, O],
                              [(0, 3, b"us"), (2, 2, None), (1, 1, None), (1, 3, b"gb")], [(0, 1, None)]),
    "Name.Url": (["Name", "Url"], [P, O], [(0, 2, b"http://A"), (1, 2, b"http://B"), (1, 1, None)],
                 [(0, 2, b"http://C")]),
}

EXPECTED_EVENTS_R1 = [  # TestColumnIO.java:114-142
    "startMessage()", "DocId.addLong(10)", "Links.start()", "Links.Forward.addLong(20)",
    "Links.Forward.addLong(40)", "Links.Forward.addLong(60)", "Links.end()", "Name.start()",
    "Name.Language.start()", "Name.Language.Code.addBinary(en-us)", "Name.Language.Country.addBinary(us)",
    "Name.Language.end()", "Name.Language.start()", "Name.Language.Code.addBinary(en)", "Name.Language.end()",
    "Name.Url.addBinary(http://A)", "Name.end()", "Name.start()", "Name.Url.addBinary(http://B)", "Name.end()",
    "Name.start()", "Name.Language.start()", "Name.Language.Code.addBinary(en-gb)",
    "Name.Language.Country.addBinary(gb)", "Name.Language.end()", "Name.end()", "endMessage()",
]


def project(events, names):
    """The events a reader of only this leaf column sees: message events, the groups on its
    path, its own values."""
    groups = {".".join(names[:k + 1]) for k in range(len(names) - 1)}
    leaf = ".".join(names)
    out = []
    for e in events:
        if e in ("startMessage()", "endMessage()"):
            out.append(e)
            continue
        head, call = e.rsplit(".", 1)
        if call in ("start()", "end()") and head in groups:
            out.append(e)
        elif head == leaf:
            out.append(e)
    return out


def stripes(rows):
    rl = [r for r, _, _ in rows]
    dl = [d for _, d, _ in rows]
    vals = [v for _, _, v in rows if v is not None]
    return rl, dl, vals


@pytest.mark.parametrize("leaf", list(PAPER))
def test_fsm_matches_expected_events_for_r1(leaf):
    names, path, r1, _ = PAPER[leaf]
    rl, dl, vals = stripes(r1)
    got = A.event_strings(path, names, A.fsm_events(path, names, rl, dl, vals))
    assert got == project(EXPECTED_EVENTS_R1, names)


def test_columnar_name_language_country():
    names, path, r1, r2 = PAPER["Name.Language.Country"]
    rl, dl, vals = stripes(r1 + r2)
    c = A.columnar(path, A.fsm_events(path, names, rl, dl, vals))
    assert c["records"] == 2
    assert c["offsets"][0] == [0, 3, 4]          # Name: 3 in r1, 1 in r2
    assert c["offsets"][1] == [0, 2, 2, 3, 3]    # Language per Name: 2, 0, 1 | 0
    assert c["validity"][2] == [1, 0, 1]         # Country per Language
    assert vals == [b"us", b"gb"]


def test_columnar_links_backward():
    names, path, r1, r2 = PAPER["Links.Backward"]
    rl, dl, vals = stripes(r1 + r2)
    c = A.columnar(path, A.fsm_events(path, names, rl, dl, vals))
    assert c["records"] == 2
    assert c["validity"][0] == [1, 1]            # Links present in both records
    assert c["offsets"][1] == [0, 0, 2]          # Backward: empty in r1, 2 values in r2
