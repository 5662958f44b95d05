"""Generate the persistent (QPB_SERVE) warm variant source of the drop-in trot
(mixed_trot_brfl golden, AMD order) wave kernel as the runtime builds it
(qpb_runtime.hip compile_variant: QPB_WARM + QPB_SERVE + kServePrelude + source),
for ISA reading on the host:

    EXTRA="#define QPB_W_EXECDBG 1" python scripts/serve_variant_src.py out.hip

COLD=1 emits the persistent cold (setup-init, QP_SETUP) variant instead.
"""
import os, re, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from apf_quadruped_amd.batch import Plan
g = np.load(os.path.join(ROOT, "tests/golden/mixed_trot_brfl.npz"))
n, m, p = int(g["n"]), int(g["m"]), int(g["p"])
print("ordering", int(g["ordering"]), n, m, p)
F = lambda M, r, c: np.asarray(M).reshape(r, c, order="F")
pl = Plan.from_dense(n, m, p, F(g["P"][0], n, n), F(g["A"][0], p, n), F(g["G"][0], m, n), kernel="wave", order="amd")
src = pl.wave_source()
rt = open(os.path.join(ROOT, "apf_quadruped_amd/csrc/qpb_runtime.hip")).read()
pre = re.search(r'kServePrelude = R"QPBS\((.*?)\)QPBS"', rt, re.S).group(1)
extra = os.environ.get("EXTRA", "")
extra = extra + "\n" if extra else ""
open(sys.argv[1], "w").write("#include <hip/hip_runtime.h>\n" + extra + ("" if os.environ.get("COLD") == "1" else "#define QPB_WARM 1\n") + "#define QPB_SERVE 1\n" + pre + src)
