"""the host-side C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only;
GPU sanitizers are not available on the GPU pool).

  * oracle/c/d2d_oracle.c (make -C oracle asan, gcc runtimes) runs tests/test_c_oracle.py: every
    env step / reset / action sampling the oracle suite drives, in-bounds and UB-free;
  * the C ABI's host code (make -C d2d-ppo_amd asan: argument checks, descriptor validation, the
    D2DEnv gather table d2d_env_single_gather_map, launch plumbing; clang runtimes, -Xarch_host
    only) runs tests/test_abi_cpu.py.
Each suite runs in a child process with the sanitizer runtime preloaded; the child first proves
that the instrumented library is the one mapped.  Leak checking is off (CPython and torch keep
allocations alive at exit) and so is the new/delete mismatch check inside uninstrumented torch."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
from sanitizer_runtimes import clang_runtime, gcc_runtimes  # noqa: E402

ENV_BASE = {"ASAN_OPTIONS": "detect_leaks=0:alloc_dealloc_mismatch=0:abort_on_error=1",
            "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "PYTHONDONTWRITEBYTECODE": "1"}


def _build(target_dir, lib):
    # incremental (a no-op when the sanitizer build is current; build() tries it up front).  Called only
    # once the runtime is known to exist, so any failure here is a build error in the host code: fail.
    r = subprocess.run(["make", "-s", "-j", str(min(8, os.cpu_count() or 2)), "-C", target_dir, "asan"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, f"sanitizer build of {target_dir} failed:\n{r.stdout[-2000:]}{r.stderr[-3000:]}"
    assert os.path.exists(lib), lib


def _run(env_extra, probe, tests):
    env = dict(os.environ)
    env.update(ENV_BASE)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", probe], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ASAN_MAPPED" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", *tests], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, r.stderr[-3000:]


def test_c_oracle_under_asan_ubsan():
    rts = gcc_runtimes()
    if rts is None:
        pytest.skip("gcc ASan / UBSan runtimes not installed on this host")
    lib = os.path.join(ROOT, "oracle", "build", "asan", "libd2d_oracle_asan.so")
    _build(os.path.join(ROOT, "oracle"), lib)
    rt = " ".join(rts)
    probe = ("import ctypes, sys; sys.path.insert(0, '.'); from oracle import c_oracle; c_oracle.lib();"
             "maps = open('/proc/self/maps').read(); assert 'libd2d_oracle_asan.so' in maps;"
             "ctypes.CDLL(None).__asan_init; print('ASAN_MAPPED')")
    _run({"D2D_ORACLE_ASAN": "1", "LD_PRELOAD": rt}, probe, ["tests/test_c_oracle.py"])


def test_abi_host_code_under_asan_ubsan():
    rt = clang_runtime()
    if rt is None:
        pytest.skip("clang ASan runtime not found under /opt/rocm/lib/llvm")
    lib = os.path.join(ROOT, "d2d-ppo_amd", "build", "asan", "libd2dhip_asan.so")
    _build(os.path.join(ROOT, "d2d-ppo_amd"), lib)
    probe = ("import ctypes, sys; sys.path[:0] = ['.', 'd2d-ppo_amd']; import d2dhip; d2dhip.load();"
             "maps = open('/proc/self/maps').read(); assert 'libd2dhip_asan.so' in maps;"
             "ctypes.CDLL(None).__asan_init; print('ASAN_MAPPED')")
    _run({"D2D_LIB_VARIANT": "asan", "LD_PRELOAD": rt}, probe, ["tests/test_abi_cpu.py"])
