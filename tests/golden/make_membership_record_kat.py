"""Writes membership_record_kat.json: the assertions of the reference's only bit-exact golden,
MembershipRecordTest (cluster/src/test/java/io/scalecube/cluster/membership/MembershipRecordTest.java:46-108),
transcribed as (r1, r0, expected isOverrides) data vectors in the packed encoding of include/swimhip.h.
r0 = null is the absent cell 0; DEAD is 0xFFFFFFFF whatever its incarnation.
"""
import json
import os

ALIVE, SUSPECT, DEAD = 1, 2, 0xFFFFFFFF


def pk(status, inc):
    return DEAD if status == DEAD else ((inc << 2) | status)


R0 = {"null": 0}
for name, st in (("Alive", ALIVE), ("Suspect", SUSPECT), ("Dead", DEAD)):
    for inc in (0, 1, 2):
        R0[f"r0{name}{inc}"] = pk(st, inc)

# (test method, r1, [(r0 name, expected)]) — one row per assertTrue/assertFalse line
CASES = [
    ("testDeadOverride", pk(DEAD, 1), [  # :47-63
        ("null", False), ("r0Alive0", True), ("r0Alive1", True), ("r0Alive2", True),
        ("r0Suspect0", True), ("r0Suspect1", True), ("r0Suspect2", True),
        ("r0Dead0", False), ("r0Dead1", False), ("r0Dead2", False)]),
    ("testAliveOverride", pk(ALIVE, 1), [  # :66-82
        ("null", True), ("r0Alive0", True), ("r0Alive1", False), ("r0Alive2", False),
        ("r0Suspect0", True), ("r0Suspect1", False), ("r0Suspect2", False),
        ("r0Dead0", False), ("r0Dead1", False), ("r0Dead2", False)]),
    ("testSuspectOverride", pk(SUSPECT, 1), [  # :85-101
        ("null", False), ("r0Alive0", True), ("r0Alive1", True), ("r0Alive2", False),
        ("r0Suspect0", True), ("r0Suspect1", False), ("r0Suspect2", False),
        ("r0Dead0", False), ("r0Dead1", False), ("r0Dead2", False)]),
]
EQUAL = [  # testEqualRecordNotOverriding :104-108
    ("r0Alive1", "r0Alive1"), ("r0Suspect1", "r0Suspect1"), ("r0Dead1", "r0Dead1")]

rows = []
for test, r1, cells in CASES:
    for r0name, exp in cells:
        rows.append({"test": test, "r1": r1, "r0": R0[r0name], "r0_name": r0name, "expected": exp})
for a, b in EQUAL:
    rows.append({"test": "testEqualRecordNotOverriding", "r1": R0[a], "r0": R0[b], "r0_name": b, "expected": False})

out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "membership_record_kat.json")
with open(out, "w") as f:
    json.dump({"source": "MembershipRecordTest.java:46-108", "rows": rows}, f, indent=1)
print(out, len(rows))
