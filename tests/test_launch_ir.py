"""Every kernel launch the host code issues survives compilation.

Round 3's host-sanitizer build launched nothing at some call sites, and
hipGetLastError said success.  Cause (scripts/micro/r3_noop_repro.sh, DESIGN.md
"Kernel launches by handle"): ``-fsanitize=function`` (part of
``-fsanitize=undefined``) instruments an indirect call's callee by reading the
8 bytes in front of it for a type signature.  A triple-chevron launch through
a kernel function pointer calls through the HIP kernel *handle*, a data
global; once inlined, that read is out of bounds of a known global, LLVM
treats the path as undefined and deletes the stub call after
``__hipPushCallConfiguration``.  The engine now launches every
function-pointer kernel by handle (hipExtLaunchKernel), and this test checks
the compiled host IR, production and sanitizer flags, for any
``__hipPushCallConfiguration`` whose launch is not reachable after it."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "kubernetes-verification_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
sys.path.insert(0, os.path.join(HERE, "tools"))

FLAGS = {
    "production": ["-O3"],
    "host-sanitizers": ["-O1", "-g0", "-Xarch_host", "-fsanitize=address", "-Xarch_host",
                        "-fsanitize=undefined", "-Xarch_host", "-fno-sanitize-recover=all"],
}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc missing")
@pytest.mark.parametrize("src", ["kano_hip.hip", "kano_ext.hip", "kano_group.hip"])
@pytest.mark.parametrize("flags", sorted(FLAGS))
def test_no_kernel_launch_dropped(src, flags, tmp_path):
    from launch_ir_check import check
    out = tmp_path / (src + ".ll")
    cmd = [HIPCC, "--offload-arch=gfx950", "-std=c++17", "--cuda-host-only", "-S", "-emit-llvm",
           *FLAGS[flags], "-I", os.path.join(ROOT, "include"), "-o", str(out),
           os.path.join(CSRC, src)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    pushes, bad = check(str(out))
    assert not bad, f"{len(bad)} of {pushes} launches dropped: {bad[:5]}"
