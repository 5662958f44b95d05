"""Host-side ISA audit: VGPRs / AGPRs live at a loop header (read on some path
before being written in the loop) and where they were last written before the loop.
A register live at the header that nothing before the loop writes carries the
previous trip's value into the next one (an undefined read on the first trip), e.g.
a value the source leaves unset in some lanes and the code reads anyway.

    python scripts/vgpr_flow.py kernel.s .LBB0_3
"""
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from sgpr_flow import parse  # noqa: E402

STORE = ("global_store", "ds_write", "buffer_store", "scratch_store", "flat_store", "global_atomic", "ds_add",
         "buffer_atomic", "flat_atomic")
SDST = ("v_cmp", "v_readlane", "v_readfirstlane", "s_")
TIED = ("v_fmac", "v_mac", "v_writelane", "v_dot2c", "v_pk_fmac")


def vregs(op):
    op = op.strip().lstrip("-|").split(" ")[0]
    m = re.fullmatch(r"([va])(\d+)", op)
    if m:
        return [m.group(1) + m.group(2)]
    m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", op)
    if m:
        return [m.group(1) + str(i) for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    return []


def defs_uses(mn, ops):
    if not ops:
        return [], []
    if mn.startswith(STORE) or mn.startswith(SDST):
        d = [] if not mn.startswith("v_cmpx") else []
        return d, [r for o in ops for r in vregs(o)]
    d = vregs(ops[0])
    u = [r for o in ops[1:] for r in vregs(o)]
    if mn.startswith(TIED):
        u += d
    return d, u


def main():
    path, header = sys.argv[1], sys.argv[2]
    blocks, order = parse(path)
    live_in = {n: set() for n in blocks}
    changed = True
    while changed:
        changed = False
        for n in reversed(order):
            live = set()
            for s in blocks[n]["succ"]:
                live |= live_in.get(s, set())
            for mn, ops, _ in reversed(blocks[n]["ins"]):
                d, u = defs_uses(mn, ops)
                live -= set(d)
                live |= set(u)
            if live != live_in[n]:
                live_in[n] = live
                changed = True
    # blocks of the loop (reachable from the header) vs before it
    seen, stack = {header}, [header]
    while stack:
        n = stack.pop()
        for s in blocks[n]["succ"]:
            if s in blocks and s not in seen:
                seen.add(s)
                stack.append(s)
    before = [n for n in order if n not in seen]
    wbefore = {}
    for n in before:
        for mn, ops, txt in blocks[n]["ins"]:
            for r in defs_uses(mn, ops)[0]:
                wbefore[r] = txt
    key = lambda r: (r[0], int(r[1:]))
    L = sorted(live_in[header], key=key)
    undef = [r for r in L if r not in wbefore]
    print(f"{len(L)} registers live at {header}; {len(undef)} with no write before the loop:")
    for r in undef:
        # first reader inside the loop
        first = None
        for n in order:
            if n not in seen:
                continue
            for mn, ops, txt in blocks[n]["ins"]:
                if r in defs_uses(mn, ops)[1]:
                    first = (n, txt)
                    break
            if first:
                break
        print(f"  {r}: first read {first}")
    for r in L:
        if r in wbefore:
            print(f"  {r}: set before the loop by `{wbefore[r]}`")


if __name__ == "__main__":
    main()
