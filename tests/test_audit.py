"""The DPP hazard audit every generated kernel with inline-asm DPP passes before
it is cached (qpb_audit_dpp, csrc/qpb_hazard.cpp): a DPP instruction must not
read ANY VGPR -- the permuted source, the other source or the tied accumulator
(the rule LLVM's checkDPPHazards applies to its own DPP code) -- written by a
VALU within 2 wait states, nor follow a VALU EXEC write within 5.  The compiler's
hazard recognizer cannot see into inline asm; the runtime compiles such kernels
through assembly and pads every DPP asm site exactly (asm_fixup), and this audit
checks the result.  CPU only (clang + llvm-objdump cross-compile and disassemble
gfx950)."""
import ctypes as C
import glob
import os
import subprocess

import pytest

from conftest import ROOT

from apf_quadruped_amd import _lib

CLANG = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin", "clang++")
SNIPPET = r"""
#include <hip/hip_runtime.h>
extern "C" __global__ void k(double *p) {
    double a = p[threadIdx.x], b = p[threadIdx.x + 64], c = p[threadIdx.x + 128];
    asm volatile("v_add_f64 %0, %0, %0\n\t" PAD "v_fmac_f64_dpp %1, %0, %2 row_newbcast:3 row_mask:0xf "
                 "bank_mask:0xf bound_ctrl:1" : "+v"(a), "+v"(c) : "v"(b));
    p[threadIdx.x] = c + a;
}
"""


def _audit(code: bytes):
    rep = C.create_string_buffer(4096)
    r = _lib.lib().qpb_audit_dpp(code, len(code), rep, 4096)
    return r, rep.value.decode()


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang not present")
@pytest.mark.parametrize("pad,expect", [("", 0), ("s_nop 0\\n\\t", 0), ("s_nop 1\\n\\t", 1),
                                        ("v_mov_b32 v200, 0\\n\\tv_mov_b32 v201, 0\\n\\t", 1)])
def test_audit_flags_dpp_source_written_too_recently(tmp_path, pad, expect):
    src = tmp_path / "k.hip"
    src.write_text(SNIPPET.replace("PAD", f'"{pad}"'))
    co = tmp_path / "k.co"
    subprocess.run([CLANG, "-x", "hip", "--cuda-device-only", "--no-gpu-bundle-output", "--offload-arch=gfx950",
                    "-O3", "-o", str(co), str(src)], check=True)
    r, rep = _audit(co.read_bytes())
    assert r == expect, rep


SNIPPET_SRC1 = r"""
#include <hip/hip_runtime.h>
extern "C" __global__ void k(double *p) {
    double a = p[threadIdx.x], b = p[threadIdx.x + 64], c = p[threadIdx.x + 128];
    asm volatile("v_add_f64 %2, %2, %2\n\t" PAD "v_fmac_f64_dpp %1, %0, %2 row_newbcast:3 row_mask:0xf "
                 "bank_mask:0xf bound_ctrl:1" : "+v"(a), "+v"(c), "+v"(b));
    p[threadIdx.x] = c + a + b;
}
"""
SNIPPET_ACC = SNIPPET_SRC1.replace('"v_add_f64 %2, %2, %2', '"v_add_f64 %1, %1, %1')


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang not present")
@pytest.mark.parametrize("snippet", ["src1", "acc"])
@pytest.mark.parametrize("pad,expect", [("", 0), ("s_nop 0\\n\\t", 0), ("s_nop 1\\n\\t", 1)])
def test_audit_flags_other_operands_written_too_recently(tmp_path, snippet, pad, expect):
    """The non-permuted source and the tied accumulator count too."""
    src = tmp_path / "k.hip"
    src.write_text((SNIPPET_SRC1 if snippet == "src1" else SNIPPET_ACC).replace("PAD", f'"{pad}"'))
    co = tmp_path / "k.co"
    subprocess.run([CLANG, "-x", "hip", "--cuda-device-only", "--no-gpu-bundle-output", "--offload-arch=gfx950",
                    "-O3", "-o", str(co), str(src)], check=True)
    r, rep = _audit(co.read_bytes())
    assert r == expect, rep


def test_cached_dpp_kernels_were_audited():
    """Every cached row / wave code object carries its audit record: clean (after
    the assembly-level padding of its DPP asm sites), or rebuilt with wait states
    in every DPP asm -- and audits clean now."""
    cache = os.path.join(ROOT, "apf_quadruped_amd", "kcache")
    objs = [f for f in glob.glob(os.path.join(cache, "qpb_row*.hsaco")) + glob.glob(os.path.join(cache, "qpb_wave*.hsaco"))]
    if not objs:
        pytest.skip("no cached kernels (run __graft_entry__.build())")
    for f in objs:
        rec = open(f + ".audit").read()
        assert rec.split("audit:")[-1].strip().startswith("clean") or "rebuilt with QPB_DPP_NOP=2" in rec, (f, rec)
        r, rep = _audit(open(f, "rb").read())
        assert r == 1 or "rebuilt" in rec, (f, rep)


TRANS_SNIPPET = r"""
#include <hip/hip_runtime.h>
extern "C" __global__ void k(double *p) {
    double a = p[threadIdx.x], b;
    asm volatile("v_rcp_f64 %0, %1\n\t" PAD "v_add_f64 %0, %0, %1" : "=&v"(b) : "v"(a));
    p[threadIdx.x] = b;
}
"""
SGPR_SNIPPET = r"""
#include <hip/hip_runtime.h>
extern "C" __global__ void k(unsigned *p) {
    unsigned v, lo = (unsigned)(size_t)p + threadIdx.x;   // (compiled and audited, never run)
    asm volatile("v_readfirstlane_b32 s60, %1\n\tv_mov_b32 %0, 0\n\ts_mov_b32 s61, 0\n\t" PAD
                 "global_load_dword %0, %0, s[60:61]\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(lo) : "s60", "s61");
    p[threadIdx.x] = v;
}
"""


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang not present")
@pytest.mark.parametrize("snippet,pad,expect", [(TRANS_SNIPPET, "", 0), (TRANS_SNIPPET, "s_nop 0\\n\\t", 1),
                                                (SGPR_SNIPPET, "", 0), (SGPR_SNIPPET, "s_nop 2\\n\\t", 1)])
def test_audit_flags_trans_forwarding_and_valu_sgpr_to_vmem(tmp_path, snippet, pad, expect):
    """Two more gfx950 hazard classes the audit checks on every instruction: a VALU
    reading a transcendental's result with no wait state between (trans forwarding,
    1 wait state), and a VMEM instruction whose SGPR base a VALU wrote within 5 wait
    states (v_readfirstlane -> global_load saddr)."""
    src = tmp_path / "k.hip"
    src.write_text(snippet.replace("PAD", f'"{pad}"'))
    co = tmp_path / "k.co"
    subprocess.run([CLANG, "-x", "hip", "--cuda-device-only", "--no-gpu-bundle-output", "--offload-arch=gfx950",
                    "-O3", "-o", str(co), str(src)], check=True)
    r, rep = _audit(co.read_bytes())
    assert r == expect, rep


def test_audit_clean_on_every_cached_kernel():
    """Every code object in the in-tree cache passes all three hazard classes
    (DPP operands / EXEC, trans forwarding, VALU SGPR -> VMEM) -- including the
    compiler-generated code around the asm."""
    objs = sorted(glob.glob(os.path.join(ROOT, "apf_quadruped_amd", "kcache", "*.hsaco")))
    if not objs:
        pytest.skip("no cached kernels (run __graft_entry__.build())")
    bad = []
    for f in objs[:400]:
        r, rep = _audit(open(f, "rb").read())
        if r == 0:
            bad.append((os.path.basename(f), rep))
    assert not bad, bad[:3]


JOIN_SNIPPET = r"""
#include <hip/hip_runtime.h>
extern "C" __global__ void k(double *p, const double *q) {
    double a = p[threadIdx.x];
    if (threadIdx.x < 6) a += q[threadIdx.x];          // divergent: s_and_saveexec / s_cbranch_execz
    p[threadIdx.x] = a * 3.0;
}
"""


def _assemble(tmp_path, text, tag):
    bindir = os.path.dirname(CLANG)
    s, o, co = tmp_path / f"{tag}.s", tmp_path / f"{tag}.o", tmp_path / f"{tag}.co"
    s.write_text(text)
    subprocess.run([os.path.join(bindir, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", str(s), "-o", str(o)], check=True)
    subprocess.run([os.path.join(bindir, "ld.lld"), "-shared", str(o), "-o", str(co)], check=True)
    return co.read_bytes()


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang not present")
def test_audit_flags_and_join_fixup_repairs_lane_partial_join(tmp_path):
    """The wide row kernel's aperture violation: the register allocator
    left `v_accvgpr_write_b32 a18, v124` (a value every lane reads later) between a
    divergent region's s_cbranch_execz target and its `s_or_b64 exec, exec, ..` restore,
    so only the region's lanes got the copy.  The same shape is injected here into a
    small kernel: the audit flags it, join_fixup moves the copy past the restore, and
    the repaired object audits clean.  (Compiled and audited, never run.)"""
    import re
    src = tmp_path / "k.hip"
    src.write_text(JOIN_SNIPPET)
    asm = tmp_path / "k.s"
    subprocess.run([CLANG, "-x", "hip", "--cuda-device-only", "--no-gpu-bundle-output", "--offload-arch=gfx950",
                    "-O3", "-S", "-o", str(asm), str(src)], check=True)
    text = asm.read_text()
    r, rep = _audit(_assemble(tmp_path, text, "clean"))
    assert r == 1, rep                                        # the compiler's own output: clean
    m = re.search(r"s_cbranch_execz (\.LBB\w+)", text)
    assert m, "no divergent region in the snippet"
    lab = m.group(1)
    bad = text.replace(f"\n{lab}:", f"\n{lab}:\n\tv_accvgpr_write_b32 a0, v0\n\ts_mov_b32 s40, s41", 1)
    assert re.search(re.escape(lab) + r":[^\n]*\n\tv_accvgpr_write_b32 a0, v0\n\ts_mov_b32 s40, s41\n(\s*;[^\n]*\n)*"
                     r"\s*s_or_b64 exec, exec", bad), "the join does not start with the EXEC restore"
    r, rep = _audit(_assemble(tmp_path, bad, "bad"))
    assert r == 0 and "1 lane-partial join(s)" in rep, rep
    buf = C.create_string_buffer(bad.encode(), len(bad) + 4096)
    jrep = C.create_string_buffer(1024)
    n = _lib.lib().qpb_join_fixup(buf, len(bad) + 4096, jrep, 1024)
    assert n == 1, jrep.value
    fixed = buf.value.decode()
    assert re.search(r"s_or_b64 exec, exec, [^\n]*\n\tv_accvgpr_write_b32 a0, v0", fixed), fixed[:3000]
    r, rep = _audit(_assemble(tmp_path, fixed, "fixed"))
    assert r == 1, rep


def test_join_fixup_refuses_a_dependent_move():
    """An instruction that reads an SGPR written after it (before the restore) cannot
    move past that write: join_fixup reports the join as not repairable (negative)."""
    text = ("k:\n\ts_and_saveexec_b64 s[0:1], vcc\n\ts_cbranch_execz .LBB0_2\n\tv_mov_b32 v1, 0\n.LBB0_2:\n"
            "\tv_mov_b32 v2, s3\n\ts_mov_b32 s3, s4\n\ts_or_b64 exec, exec, s[0:1]\n\ts_endpgm\n")
    buf = C.create_string_buffer(text.encode(), len(text) + 1024)
    jrep = C.create_string_buffer(1024)
    assert _lib.lib().qpb_join_fixup(buf, len(text) + 1024, jrep, 1024) == -1, jrep.value
    ok = text.replace("\tv_mov_b32 v2, s3\n\ts_mov_b32 s3, s4\n", "\tv_mov_b32 v2, s5\n\ts_mov_b32 s3, s4\n")
    buf = C.create_string_buffer(ok.encode(), len(ok) + 1024)
    assert _lib.lib().qpb_join_fixup(buf, len(ok) + 1024, jrep, 1024) == 1, jrep.value
    assert "s_or_b64 exec, exec, s[0:1]\n\tv_mov_b32 v2, s5" in buf.value.decode()


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not present")
@pytest.mark.parametrize("src", ["qpb_comm.hip", "qpb_assemble.hip", "qpb_runtime.hip"])
def test_static_device_code_passes_the_audit(tmp_path, src):
    """The kernels compiled into libqpswift_hip.so itself (argmin, winner payload, strided
    copies, assembly, the RCCL gather's device reduce) pass the same code-object audit as
    the generated ones -- in particular no lane-masked copy ahead of an EXEC restore."""
    co = tmp_path / "k.co"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "--cuda-device-only",
                    "--no-gpu-bundle-output", "-o", str(co), os.path.join(ROOT, "apf_quadruped_amd", "csrc", src)],
                   check=True, capture_output=True)
    r, rep = _audit(co.read_bytes())
    assert r == 1, rep
