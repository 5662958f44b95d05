"""Host-side ISA audit of SGPR spills to VGPR lanes: on every path from the kernel's
entry to a `v_readlane_b32 sX, vN, L`, has lane L of vN been written by a
`v_writelane_b32 vN, sY, L` (and by nothing else since)?  A reload on a path that
skips the spill returns whatever the VGPR lane held -- for kernarg pointers parked
there, a garbage 64-bit address (HSA memory-aperture violation).

Works on `llvm-objdump -d --mcpu=gfx950` output of one kernel.  Must-analysis over the
basic blocks (intersection at joins); a VALU write of the whole VGPR (any other
instruction naming it as destination) kills every lane.

    python scripts/spill_lane_audit.py kernel.hsaco [vgpr]
"""
import re
import subprocess
import sys

LINE = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
TGT = re.compile(r"<[^+>]+\+0x([0-9a-f]+)>")


def disasm(path):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", path],
                         capture_output=True, text=True, check=True).stdout
    ins, base = [], None
    for ln in out.split("\n"):
        m = re.match(r"^([0-9a-f]+) <([^>]+)>:", ln)
        if m:
            base = int(m.group(1), 16)
            continue
        m = LINE.match(ln)
        if m and base is not None:
            op, args, addr = m.group(1), m.group(2), int(m.group(3), 16)
            t = TGT.search(ln)
            ins.append((addr, op, args, base + int(t.group(1), 16) if t else None))
    return ins


def audit(ins, vreg):
    addrs = [a for a, *_ in ins]
    idx = {a: i for i, a in enumerate(addrs)}
    # leaders
    lead = {0}
    for i, (a, op, args, tgt) in enumerate(ins):
        if op.startswith("s_branch") or op.startswith("s_cbranch"):
            if tgt is not None and tgt in idx:
                lead.add(idx[tgt])
            lead.add(i + 1)
        if op == "s_endpgm":
            lead.add(i + 1)
    lead = sorted(x for x in lead if x < len(ins))
    blocks = []
    for k, s in enumerate(lead):
        e = lead[k + 1] if k + 1 < len(lead) else len(ins)
        blocks.append((s, e))
    bof = {s: k for k, (s, e) in enumerate(blocks)}
    succ = []
    for s, e in blocks:
        a, op, args, tgt = ins[e - 1]
        ss = []
        if op.startswith("s_branch"):
            ss.append(bof[idx[tgt]])
        elif op.startswith("s_cbranch"):
            ss.append(bof[idx[tgt]])
            if e < len(ins):
                ss.append(bof[e])
        elif op != "s_endpgm" and e < len(ins):
            ss.append(bof[e])
        succ.append(ss)
    wl = re.compile(r"^%s,\s*\S+,\s*(\d+)$" % re.escape(vreg))
    rl = re.compile(r"^\S+,\s*%s,\s*(\d+)$" % re.escape(vreg))
    dst_kill = re.compile(r"^(%s\b|v\[(\d+):(\d+)\])" % re.escape(vreg))
    vn = int(vreg[1:])

    def transfer(st, i, report=None):
        a, op, args, tgt = ins[i]
        if op == "v_writelane_b32":
            m = wl.match(args)
            if m:
                return st | {int(m.group(1))}
        if op == "v_readlane_b32":
            m = rl.match(args)
            if m and report is not None and int(m.group(1)) not in st:
                report.append((a, op, args))
            return st
        if op.startswith("v_") or op.startswith("ds_read") or op.startswith("global_load") \
                or op.startswith("buffer_load") or op.startswith("scratch_load") or op.startswith("flat_load"):
            m = dst_kill.match(args)
            if m:
                if m.group(2) is None or int(m.group(2)) <= vn <= int(m.group(3)):
                    return frozenset()
        return st

    ALL = frozenset(range(64))
    inn = [ALL] * len(blocks)
    inn[0] = frozenset()
    outs = [ALL] * len(blocks)
    changed = True
    while changed:
        changed = False
        for k, (s, e) in enumerate(blocks):
            st = inn[k]
            for i in range(s, e):
                st = transfer(st, i)
            if st != outs[k]:
                outs[k] = st
                changed = True
            for t in succ[k]:
                nv = inn[t] & st if t != 0 else frozenset()
                if nv != inn[t]:
                    inn[t] = nv
                    changed = True
    bad = []
    for k, (s, e) in enumerate(blocks):
        st = inn[k]
        for i in range(s, e):
            st = transfer(st, i, bad)
    return bad, len(blocks)


def main():
    path = sys.argv[1]
    vreg = sys.argv[2] if len(sys.argv) > 2 else "v255"
    ins = disasm(path)
    bad, nb = audit(ins, vreg)
    print(f"{path}: {len(ins)} instructions, {nb} blocks, {vreg}: "
          f"{len(bad)} reload(s) reachable without their spill")
    for a, op, args in bad:
        print(f"  0x{a:X}: {op} {args}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
