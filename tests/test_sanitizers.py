"""Host sanitizers ("build host code with ASan/UBSan"): the
oracle (CPU) and the engine's host code through its C ABI (the device code
is built normally: -Xarch_host), both built by __graft_entry__.build().
tests/asan/kano_asan.cpp checks the engine against a naive restatement of
build_matrix and the checks and walks the ABI's error paths, row shards,
incremental updates and row digests; ASan / UBSan abort on any memory or
undefined-behaviour error in the host code."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:abort_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _run(path, timeout):
    assert os.path.exists(path), f"{path} missing: run __graft_entry__.build()"
    return subprocess.run([path], capture_output=True, text=True, timeout=timeout, env=ENV)


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True,
                   capture_output=True)
    r = _run(os.path.join(ROOT, "oracle", "_asan", "oracle_asan"), 120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "clean" in r.stdout


def test_engine_host_asan_without_device():
    """Without a GPU the sanitized engine reports -ENODEV and exits 77."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: the -m gpu test runs the full driver")
    r = _run(os.path.join(HERE, "asan", "kano_asan"), 120)
    assert r.returncode == 77, r.stdout + r.stderr


@pytest.mark.gpu
def test_engine_host_under_asan_ubsan():
    # (ASan's quarantine stays on -- use-after-free in the engine's host code
    # is caught; the driver ends with _Exit after its checks, so the HIP
    # runtime's static teardown does not recycle quarantined allocations)
    env = ENV
    path = os.path.join(HERE, "asan", "kano_asan")
    assert os.path.exists(path), f"{path} missing: run __graft_entry__.build()"
    r = subprocess.run([path], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert r.stdout.startswith("ok"), r.stdout
