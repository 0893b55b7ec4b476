"""The compiler behaviour behind round 5's wrong row-staged data gradients, on the CPU (no GPU): hipcc
(ROCm 7.2) lowers `__builtin_bit_cast(unsigned, acc[j][r])` — a bit cast of an ext_vector component
lvalue — to a copy of component 0, so the unrolled epilogue stores ONE register per accumulator for all
16 r; casting the component to a value first (the product form) stores 16 distinct registers.  Reads the
device ISA of csrc/diag.hip's two variants (csrc/diag.hip, tests/test_diag_gpu.py)."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_component_bitcast_store_isa(tmp_path):
    out = tmp_path / "diag.s"
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-I", os.path.join(REPO, "include"),
                        os.path.join(REPO, "speechrecognitionproject_amd", "csrc", "diag.hip"), "-o", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    s = out.read_text()
    srcs = {}
    for v in ("0", "1"):
        m = re.search(r"acc_store_kernelILi%sEEEvPfi:(.*?)s_endpgm" % v, s, re.S)
        assert m, v
        srcs[v] = re.findall(r"buffer_store_dword ([av]\d+)", m.group(1))
        assert len(srcs[v]) == 32, (v, len(srcs[v]))
    assert len(set(srcs["0"])) == 32          # the product form: every accumulator register stored
    # the round-5 form: the two accumulators' component 0 only (if a later compiler fixes the lowering,
    # this is where it shows)
    assert len(set(srcs["1"])) == 2
