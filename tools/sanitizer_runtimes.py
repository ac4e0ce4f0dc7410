"""Sanitizer runtime probes shared by __graft_entry__.build() and tests/test_sanitizers_cpu.py.
Standard library only (no pytest / numpy), so the product build does not depend on the test
requirements; a host without gcc or the ROCm clang runtime reports "no runtime" (None)."""
import glob
import os
import subprocess


def gcc_runtimes():
    """The gcc ASan / UBSan runtimes (the C oracle's), or None when this host has none (or no gcc)."""
    try:
        paths = [subprocess.run(["gcc", f"-print-file-name={n}"], capture_output=True, text=True).stdout.strip()
                 for n in ("libasan.so", "libubsan.so")]
    except (FileNotFoundError, PermissionError):
        return None
    return paths if all(os.path.isabs(p) and os.path.exists(p) for p in paths) else None


def clang_runtime():
    """The clang ASan runtime of the ROCm toolchain (the HIP library's host code), or None."""
    rts = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    return rts[0] if rts else None
