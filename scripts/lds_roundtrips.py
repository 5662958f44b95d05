"""Count "lone" LDS round trips in a code object's disassembly: an `s_waitcnt lgkmcnt(0)`
whose window since the previous wait holds exactly one LDS read, i.e. a load the wave
waits for by itself (~120 cycles on the chain) instead of in a batch.  Round 6 found
the register allocator serialising loads this way in the row kernel's prologue, the wide
row kernel's H0 staging, the wave kernel's residual / solve products and the band
kernel's per-row passes.

    python scripts/lds_roundtrips.py KERNEL.hsaco [...]      (-v: list the sites)
"""
import re
import subprocess
import sys

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def disasm(path):
    txt = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", path], capture_output=True, text=True, check=True).stdout
    ins = []
    for line in txt.splitlines():
        m = re.match(r"\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return ins


def loops(ins):
    out = []
    for a, mn, ops in ins:
        if mn.startswith("s_branch") or mn.startswith("s_cbranch"):
            v = int(ops.split()[0])
            v = v - 65536 if v > 32767 else v
            t = a + 4 + 4 * v
            if t < a:
                out.append((t, a))
    return out


def lone_sites(ins):
    sites = []
    for i, (a, mn, ops) in enumerate(ins):
        if mn == "s_waitcnt" and "lgkmcnt(0)" in ops:
            j, reads = i - 1, []
            while j >= 0 and ins[j][1] != "s_waitcnt":
                if ins[j][1].startswith("ds_read"):
                    reads.append(j)
                j -= 1
            if len(reads) == 1:
                sites.append((i, reads[0]))
    return sites


def main():
    verbose = "-v" in sys.argv
    for path in [p for p in sys.argv[1:] if p != "-v"]:
        ins = disasm(path)
        lp = loops(ins)
        sites = lone_sites(ins)
        waits = sum(1 for _, mn, o in ins if mn == "s_waitcnt" and "lgkmcnt(0)" in o)
        print(f"{path}: {len(sites)} lone LDS round trips of {waits} lgkmcnt(0) waits, {len(ins)} instructions")
        if verbose:
            for w, r in sites:
                a, mn, ops = ins[r]
                inner = [f"{t:#x}-{e:#x}" for t, e in lp if t <= ins[w][0] <= e and e - t < 4096]
                print(f"  wait at {ins[w][0]:#x}: {mn} {ops[:48]}" + (f"  (loop {inner[0]})" if inner else ""))


if __name__ == "__main__":
    main()
