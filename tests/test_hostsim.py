"""CPU test: the library's host runtime under AddressSanitizer, with HIP replaced by a host stand-in
(tests/hostsim/hip_stub.cpp). Exercises descriptor validation, staging, group-by key decoding and
result assembly for every known-answer query without a GPU."""
import os
import subprocess
import sys

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hostsim")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(HERE, "libpinot_hip_hostsim.so")
ASAN = "/opt/rocm/lib/llvm/lib/clang/22/lib/linux/libclang_rt.asan-x86_64.so"


def _build():
    src = [os.path.join(ROOT, "pinot_amd", "csrc", "runtime.cpp"), os.path.join(ROOT, "pinot_amd", "csrc", "node.cpp"),
           os.path.join(HERE, "hip_stub.cpp")]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-host-only", "-O1", "-g", "-std=c++17", "-fPIC", "-shared",
                           "-fsanitize=address", "-fno-omit-frame-pointer", "-nogpulib", "-o", SO] + src + ["-ldl"],
                          stderr=subprocess.DEVNULL)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or not os.path.exists(ASAN), reason="needs hipcc + ASan runtime")
def test_host_runtime_under_asan():
    _build()
    env = dict(os.environ, LD_PRELOAD=ASAN, ASAN_OPTIONS="detect_leaks=0")
    p = subprocess.run([sys.executable, os.path.join(HERE, "run_host_paths.py"), SO], env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0 and "HOSTSIM OK" in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or not os.path.exists(ASAN), reason="needs hipcc + ASan runtime")
@pytest.mark.parametrize("ndev", [2, 3])
def test_node_plans_under_asan(ndev):
    """Node plans (node.cpp) over segments on 2 / 3 stand-in devices: the sub-plans' descriptors, the peer-merge
    exchange (whose merged count proves every part's table was folded in), the record merge and the refusals."""
    if not os.path.exists(SO):
        _build()
    env = dict(os.environ, LD_PRELOAD=ASAN, ASAN_OPTIONS="detect_leaks=0", HOSTSIM_DEVICES=str(ndev))
    p = subprocess.run([sys.executable, os.path.join(HERE, "run_node_paths.py"), SO], env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0 and "HOSTSIM NODE OK" in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]
