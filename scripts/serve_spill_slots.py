"""Resident-solver diagnostics (DESIGN_HISTORY §4i): SGPR spill slots (v254/v255 lanes)
written before the request loop and rewritten inside it (clang -S output of
scripts/serve_variant_src.py)."""
import re, sys
L = open(sys.argv[1]).read().split("\n")
inloop = False; cur = None
pre = {}; loopw = {}; loopr = {}
for i, l in enumerate(L):
    m = re.match(r"^(\.LBB0_\d+|; %bb\.\d+):?\s*(;.*)?$", l.strip())
    if m:
        c = l
        inloop = ("Header=BB0_3" in c) or ("This Loop Header: Depth=1" in c) or ("Parent Loop BB0_3" in c)
        if "s_endpgm" in c: inloop = False
        continue
    m = re.match(r"\s*v_writelane_b32 (v25[45]), (s\d+), (\d+)", l)
    if m:
        key = (m.group(1), int(m.group(3)))
        (loopw if inloop else pre).setdefault(key, []).append(i + 1)
    m = re.match(r"\s*v_readlane_b32 (s\d+), (v25[45]), (\d+)", l)
    if m and inloop:
        loopr.setdefault((m.group(2), int(m.group(3))), []).append(i + 1)
both = sorted(set(pre) & set(loopw))
print("slots written before the loop:", len(pre), " inside:", len(loopw), " both:", both)
for k in both:
    print(k, "pre", pre[k][:3], "loop writes", loopw[k][:5], "loop reads", loopr.get(k, [])[:5])
