"""Where a code object's DPP wait states go: every `s_nop` in front of a DPP instruction,
classified by the operand whose recent VALU write it waits out -- `src0` (the broadcast
source: chains such as the triangular solves, inherent), `acc` (the accumulator written
by one of the two previous instructions), `src1` (the multiplier, e.g. a product formed
right before the FMAs that read it: the wide row GᵀWG before round 6's one-row-behind
order) -- and by the producing instruction.  Static counts over the object.

    python scripts/dpp_wait_states.py KERNEL.hsaco [...]
"""
import collections
import re
import subprocess
import sys

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def disasm(path):
    txt = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", path], capture_output=True, text=True, check=True).stdout
    out = []
    for line in txt.splitlines():
        m = re.match(r"\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
        if m:
            out.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return out


def vregs(op):
    out = []
    for r in re.findall(r"v\[(\d+):(\d+)\]|v(\d+)", op):
        out.append((int(r[2]), int(r[2])) if r[2] else (int(r[0]), int(r[1])))
    return out


def classify(ins):
    overlap = lambda a, b: a is not None and b is not None and a[0] <= b[1] and b[0] <= a[1]
    sites, states = collections.Counter(), collections.Counter()
    for i, (_, mn, ops) in enumerate(ins):
        if mn != "s_nop" or i + 1 >= len(ins) or "dpp" not in ins[i + 1][1]:
            continue
        fields = [x.strip() for x in ins[i + 1][2].split(",")]
        regs = [vregs(f)[0] if vregs(f) else None for f in fields[:3]] + [None] * 3
        dst, src0, src1 = regs[0], regs[1], regs[2]
        why, prod = "other", None
        for j in range(i - 1, max(i - 4, -1), -1):
            pm, po = ins[j][1], ins[j][2]
            if not pm.startswith("v_"):
                continue
            pd = vregs(po.split(",")[0])
            if not pd:
                continue
            if overlap(pd[0], src0):
                why, prod = "src0", pm
            elif overlap(pd[0], dst):
                why, prod = "acc", pm
            elif overlap(pd[0], src1):
                why, prod = "src1", pm
            else:
                continue
            break
        sites[(why, prod)] += 1
        states[(why, prod)] += int(ops.split()[0]) + 1
    return sites, states


def main():
    for path in sys.argv[1:]:
        sites, states = classify(disasm(path))
        print(f"{path}: {sum(sites.values())} DPP instructions behind an s_nop, {sum(states.values())} wait states")
        for key, n in sites.most_common(8):
            print(f"  {n:4d} sites {states[key]:4d} wait states  {key[0]:5s} written by {key[1]}")


if __name__ == "__main__":
    main()
