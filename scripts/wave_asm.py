"""Dump the generated wave-kernel source for a standard shape and compile it to
gfx950 assembly with hipcc (same flags as the hiprtc JIT), for ISA reading.

    QPB_WAVE_OPTS="QPB_W_TIMING=1" python scripts/wave_asm.py [c1|c30][:amd] [out_prefix]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "c1"
    shape, _, order = shape.partition(":")       # "c30:amd": the AMD-ordered plan
    out = sys.argv[2] if len(sys.argv) > 2 else f"/tmp/wave_{shape}"
    from apf_quadruped_amd import plans
    from apf_quadruped_amd.batch import Plan
    from apf_quadruped_amd import workloads as W
    if shape == "c1":
        d = plans.standard_qp("c1")
        pl = Plan.from_dense(12, 20, 6, d["P"][0], d["A"][0], d["G"][0], kernel="wave", order=order or "own")
    else:
        d = W.controller_qp(plans.SEED + 30, [0])
        pl = Plan.from_dense(d["n"], d["m"], d["p"], d["P"][0], d["A"][0], d["G"][0], kernel="wave",
                             order=order or "own")
    src = "#include <hip/hip_runtime.h>\n" + pl.wave_source()
    open(out + ".hip", "w").write(src)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "--cuda-device-only", "-S", "-o", out + ".s", out + ".hip"])
    print(out + ".s")


if __name__ == "__main__":
    main()
