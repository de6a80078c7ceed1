"""Debug helper: diff one golden case's GPU matches against the fixture."""
import json, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import ugrep_amd as U
from oracle_lib import case_input
pats = json.load(open("tests/golden/patterns.json"))
cases = json.load(open("tests/golden/cases.json"))
pn, name = sys.argv[1], sys.argv[2]
c = [c for c in cases if c["pattern"] == pn and c["input"].get("name") == name][0]
data = case_input(c["input"])
r = U.find_all(U.Pattern(pats[pn]["opc"]), data.tobytes(), offsets=True)
got = r.triples()
exp = c["matches"]
print("n", len(data), "got", len(got), "exp", len(exp))
sg, se = set(map(tuple, got)), set(map(tuple, exp))
print("missing", sorted(se - sg)[:20])
print("extra", sorted(sg - se)[:20])
