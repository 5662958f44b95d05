"""Host-side ISA audit for VALU code placed between a divergent region's skip target and
its EXEC restore.

LLVM lowers `if (divergent) {...}` to
    s_and_saveexec_b64 s[a:b], cond ; s_cbranch_execz JOIN ; <then> ; JOIN: s_or_b64 exec, exec, s[a:b]
When the execz branch is taken no lane is active, so anything placed at JOIN *before*
the `s_or_b64 exec` restore runs with the then-region's partial EXEC.  The register
allocator treats JOIN as the join block (all lanes), so a copy it inserts there -- a
VGPR parked in an AGPR, a live-range split -- is made only for the then-lanes; the
other lanes later read a stale register.  This found the wide row kernel's
memory-aperture violation: `tile` copied to a18:a19 under the `c < NY`
mask of the b-vector load, read by every lane to form the z / s output addresses.

    python scripts/exec_join_audit.py kernel.hsaco [...]

The same check runs inside the library on every kernel it builds (qpb_audit_dpp,
csrc/qpb_hazard.cpp); this script is the standalone form for cached objects.
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
            t = TGT.search(ln)
            ins.append((int(m.group(3), 16), m.group(1), m.group(2),
                        base + int(t.group(1), 16) if t else None))
    return ins


def writes_exec(op, args):
    return args.startswith("exec") or "saveexec" in op or op.startswith("v_cmpx")


def audit(ins):
    idx = {a: i for i, (a, *_) in enumerate(ins)}
    bad = []
    for i, (a, op, args, tgt) in enumerate(ins):
        if op != "s_cbranch_execz" or tgt not in idx:
            continue
        j = idx[tgt]
        found = []
        while j < len(ins):
            a2, op2, args2, _ = ins[j]
            if writes_exec(op2, args2) or op2.startswith("s_branch") or op2.startswith("s_cbranch") \
                    or op2 == "s_endpgm":
                break
            if op2.startswith(("v_", "ds_", "global_", "buffer_", "flat_", "scratch_")) \
                    and not op2.startswith(("v_readlane", "v_readfirstlane", "v_writelane", "v_cmp_")) \
                    and not op2.startswith(("global_store", "buffer_store", "ds_write", "flat_store", "scratch_store")):
                found.append((a2, op2, args2))
            j += 1
        # only a JOIN whose first exec write is the restore `s_or_b64 exec, exec, ...`
        if found and j < len(ins) and ins[j][1] == "s_or_b64" and ins[j][2].startswith("exec, exec"):
            bad.append((a, tgt, ins[j][0], found))
    return bad


def main():
    rc = 0
    for path in sys.argv[1:]:
        bad = audit(disasm(path))
        print(f"{path}: {len(bad)} join(s) with lane-partial code before the EXEC restore")
        for a, tgt, rst, found in bad:
            rc = 1
            print(f"  execz at 0x{a:X} -> 0x{tgt:X}, restore at 0x{rst:X}:")
            for a2, op2, args2 in found:
                print(f"    0x{a2:X}: {op2} {args2}")
    return rc


if __name__ == "__main__":
    sys.exit(main())
