"""Host-side ISA audit: may an SGPR's value entering a loop differ from what the
preheader set?  Forward dataflow over the basic blocks of one kernel's clang -S output,
tracking the value of each watched SGPR symbolically (copies between registers are
followed; every other write makes it unknown).  Reports, for each loop header label,
the watched registers that can arrive there with a value other than the preheader's.

    python scripts/sgpr_flow.py kernel.s .LBB0_3 [s15 s71 ...]

With no register list every SGPR written before the header is watched; only the
registers live at the header (read before written on some path) are reported.
"""
import re
import sys

BR = re.compile(r"^\s+s_branch\s+(\.LBB\w+)")
CBR = re.compile(r"^\s+s_cbranch_\w+\s+(\.LBB\w+)")
LABEL = re.compile(r"^(\.LBB\w+):")
BB = re.compile(r"^; %bb\.(\d+):")
INS = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*))?$")
NODEST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_sleep", "s_endpgm", "global_store",
          "ds_write", "buffer_store", "buffer_inv", "buffer_wbl2", "scratch_store", "flat_store", "s_setprio",
          "s_barrier", "s_store", "ds_read_addtid", "s_trap", "s_dcache", "s_icache", "v_cmp_", "v_cmpx_")


def regs(op):
    """The SGPR numbers an operand names (s7, s[4:5]); vcc / exec excluded."""
    m = re.fullmatch(r"s(\d+)", op)
    if m:
        return [int(m.group(1))]
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", op)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return []


def parse(path, kernel=None):
    lines = open(path).read().split("\n")
    blocks, cur, order = {}, None, []
    for ln in lines:
        if ln.startswith("\t.size") or ln.startswith("\t.end_amdhsa"):
            cur = None
        m = LABEL.match(ln) or BB.match(ln)
        if m:
            name = m.group(1) if ln.startswith(".") else "%bb." + m.group(1)
            if cur is not None and not blocks[cur]["term"]:
                blocks[cur]["succ"].append(name)
            cur = name
            blocks[cur] = {"ins": [], "succ": [], "term": False}
            order.append(cur)
            continue
        if cur is None:
            if ln.strip().endswith(":") and not ln.startswith("\t") and not ln.startswith("."):
                cur = "entry"
                blocks[cur] = {"ins": [], "succ": [], "term": False}
                order.append(cur)
            continue
        if blocks[cur]["term"]:
            continue
        m = INS.match(ln)
        if not m or ln.lstrip().startswith(";") or ln.lstrip().startswith("."):
            continue
        mn, rest = m.group(1), (m.group(2) or "").split(";")[0]
        ops = [o.strip() for o in rest.split(",")] if rest.strip() else []
        blocks[cur]["ins"].append((mn, ops, ln.strip()))
        b = BR.match(ln)
        if b:
            blocks[cur]["succ"].append(b.group(1))
            blocks[cur]["term"] = True
        c = CBR.match(ln)
        if c:
            blocks[cur]["succ"].append(c.group(1))
        if mn == "s_endpgm":
            blocks[cur]["term"] = True
    # fallthrough from a block that did not end in an unconditional branch
    for i, name in enumerate(order[:-1]):
        b = blocks[name]
        if not b["term"] and order[i + 1] not in b["succ"]:
            b["succ"].append(order[i + 1])
    return blocks, order


def dests(mn, ops):
    if not ops or any(mn.startswith(p) for p in NODEST):
        # v_cmp_*_e64 writes its first (SGPR pair) operand
        if mn.startswith("v_cmp") and mn.endswith("_e64") and ops:
            return regs(ops[0])
        return []
    return regs(ops[0])


def lane_key(v, n):
    """An SGPR spill lane (v_writelane / v_readlane of a VGPR) as a pseudo-register."""
    return 1000 * (int(v[1:]) + 1) + int(n)


def transfer(state, ins):
    st = dict(state)
    for mn, ops, _ in ins:
        if mn == "v_writelane_b32" and len(ops) == 3 and regs(ops[1]) and ops[2].isdigit():
            st[lane_key(ops[0], ops[2])] = st.get(regs(ops[1])[0], ("init", regs(ops[1])[0]))
            continue
        if mn == "v_readlane_b32" and len(ops) == 3 and regs(ops[0]) and ops[2].isdigit() and ops[1].startswith("v"):
            k = lane_key(ops[1], ops[2])
            st[regs(ops[0])[0]] = st.get(k, ("init", k))
            continue
        ds = dests(mn, ops)
        if not ds:
            continue
        if mn == "s_mov_b32" and len(ops) == 2 and regs(ops[1]) and len(ds) == 1:
            src = regs(ops[1])[0]
            st[ds[0]] = st.get(src, ("init", src))
            continue
        if mn == "s_mov_b64" and len(ops) == 2 and len(regs(ops[1])) == 2 and len(ds) == 2:
            s = regs(ops[1])
            v = [st.get(r, ("init", r)) for r in s]
            st[ds[0]], st[ds[1]] = v
            continue
        if mn == "s_mov_b32" and len(ops) == 2 and re.fullmatch(r"-?(0x[0-9a-f]+|\d+)", ops[1]):
            for d in ds:
                st[d] = ("const", int(ops[1], 0))
            continue
        for d in ds:
            st[d] = ("unknown",)
    return st


def main():
    path, header = sys.argv[1], sys.argv[2]
    watch = [int(r[1:]) for r in sys.argv[3:]]
    blocks, order = parse(path)
    preds = {n: [] for n in blocks}
    for n, b in blocks.items():
        for s in b["succ"]:
            if s in preds:
                preds[s].append(n)
    # state at the end of each block; values are ("init", r) at kernel entry
    out = {n: None for n in blocks}
    TOP = None

    def join(a, b):
        if a is TOP:
            return b
        res = {}
        for k in set(a) | set(b):
            va, vb = a.get(k, ("init", k)), b.get(k, ("init", k))
            res[k] = va if va == vb else ("unknown",)
        return res

    changed = True
    while changed:
        changed = False
        for n in order:
            ins = TOP
            if n == order[0]:
                ins = {}
            for p in preds[n]:
                if out[p] is not TOP:
                    ins = join(ins, out[p])
            if ins is TOP:
                continue
            o = transfer(ins, blocks[n]["ins"])
            if o != out[n]:
                out[n] = o
                changed = True
    # the header: preheader (non-loop) edge vs back edges
    hp = preds[header]
    seen, stack = set(), [header]
    while stack:
        n = stack.pop()
        for s in blocks[n]["succ"]:
            if s in blocks and s not in seen:
                seen.add(s)
                stack.append(s)
    back = [p for p in hp if p in seen]       # in the loop: reachable from the header
    pre = [p for p in hp if p not in seen]
    sp = TOP
    for p in pre:
        sp = join(sp, out[p])
    # live SGPRs at the header (read on some path before being written)
    def uses(mn, ops):
        d = dests(mn, ops)
        src = ops[1:] if d else ops
        return [r for o in src for r in regs(o.split(" ")[0])]

    live_in = {n: set() for n in blocks}
    changed = True
    while changed:
        changed = False
        for n in reversed(order):
            live = set()
            for sname in blocks[n]["succ"]:
                live |= live_in.get(sname, set())
            for mn, ops, _ in reversed(blocks[n]["ins"]):
                if mn == "v_writelane_b32" and len(ops) == 3 and ops[2].isdigit():
                    live.discard(lane_key(ops[0], ops[2]))
                    live |= set(regs(ops[1]))
                    continue
                if mn == "v_readlane_b32" and len(ops) == 3 and ops[2].isdigit() and ops[1].startswith("v"):
                    live -= set(regs(ops[0]))
                    live.add(lane_key(ops[1], ops[2]))
                    continue
                live -= set(dests(mn, ops))
                live |= set(uses(mn, ops))
            if live != live_in[n]:
                live_in[n] = live
                changed = True
    lanes = sorted(k for k in live_in[header] if k >= 1000)
    regs_w = [r for r in (watch or sorted(k for k in sp if isinstance(k, int))) if r in live_in[header]] + lanes
    print(f"live at {header}: {sorted(live_in[header])}")
    print(f"{header}: preheaders {pre}, back edges {back}")
    bad = 0
    for r in regs_w:
        v0 = sp.get(r, ("init", r))
        for p in back:
            v = out[p].get(r, ("init", r)) if out[p] else None
            if v != v0:
                bad += 1
                nm = f"s{r}" if r < 1000 else f"v{r // 1000 - 1} lane {r % 1000}"
                print(f"  {nm}: enters as {v0}, back edge from {p} brings {v}")
    print(f"{bad} mismatching (register, back edge) pairs")


if __name__ == "__main__":
    main()
