"""Static hazard check of the hand-written DPP FMAs (fmac_bc, csrc/qpb_common.h).

gfx950 needs two wait states between a VALU write of a VGPR and a DPP read of
it; hipcc does not pad inline asm.  tools/check_dpp_hazards.py walks every
path into every DPP instruction of libqpb's device code (CPU only: it reads
the gfx950 code objects inside build/*.o with llvm-objdump).
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "embedded-qp-solver_amd", "build")
TOOL = os.path.join(ROOT, "tools", "check_dpp_hazards.py")
HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

pytestmark = pytest.mark.skipif(not (os.path.exists(OBJDUMP) and glob.glob(os.path.join(BUILD, "qpb_*.o"))),
                                reason="needs the ROCm llvm tools and the built objects (make -C embedded-qp-solver_amd)")


def _run(build):
    return subprocess.run([sys.executable, TOOL, build], capture_output=True, text=True)


def test_library_has_no_dpp_read_hazard(tmp_path):
    # only the library's own objects (A/B variant objects may sit beside them)
    for o in glob.glob(os.path.join(BUILD, "qpb_*.o")):
        os.symlink(o, tmp_path / os.path.basename(o))
    r = _run(str(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 hazards" in r.stdout


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc")
def test_checker_flags_a_deliberate_hazard(tmp_path):
    src = tmp_path / "hz.hip"
    src.write_text(
        '#include "qpb_common.h"\n'
        "__global__ void hz(double *p) {\n"
        "  double a = p[threadIdx.x], b = p[threadIdx.x + 64], acc = 0.0;\n"
        "  double v = a * b;\n"
        "  qpb::fmac_bc<3>(acc, v, b);  // no wait states after v's producer\n"
        "  p[threadIdx.x] = acc;\n"
        "}\n")
    subprocess.run([HIPCC, "-std=c++20", "-O3", "--offload-arch=gfx950",
                    "-I" + os.path.join(ROOT, "embedded-qp-solver_amd", "csrc"), "-c", str(src), "-o",
                    str(tmp_path / "hz.o")], check=True, capture_output=True)
    r = _run(str(tmp_path))
    assert r.returncode == 1 and " 1 hazards" in r.stdout, r.stdout
