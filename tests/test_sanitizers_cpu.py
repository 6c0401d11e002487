"""Host C++ runtime (``csrc/runtime``: DAG programs, CSR build, synthetic graphs and
shards, the locality reorder, the host neighbour sampler) under AddressSanitizer +
UndefinedBehaviorSanitizer: a sanitized build of ``_rt`` is loaded in place of the
normal one (``CGNN_RT_LIB``) and the runtime's CPU test files run against it; any
ASan report or UBSan runtime error aborts the run.  (GPU code cannot be sanitized on
this pool; its checks are the oracle tests.)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gcc_lib(name):
    out = subprocess.run(["g++", "-print-file-name=" + name], stdout=subprocess.PIPE, text=True)
    path = out.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def _libasan():
    return _gcc_lib("libasan.so")


def test_runtime_under_address_and_ub_sanitizers(tmp_path):
    import pytest
    from cgnn_amd import _build
    asan = _libasan()
    if asan is None:
        pytest.skip("no libasan for the host compiler")
    target = str(tmp_path / ("_rt" + _build.EXT))
    _build.build_rt(force=True, debug=True, target=target)
    # libstdc++ preloaded right after ASan: python itself does not link it, and ASan's
    # __cxa_throw interceptor must resolve the real one when the runtime throws (a
    # rejected argument), or the process aborts in the interceptor
    pre = asan + (":" + _gcc_lib("libstdc++.so") if _gcc_lib("libstdc++.so") else "")
    env = dict(os.environ, LD_PRELOAD=pre, CGNN_RT_LIB=target,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="4")
    probe = subprocess.run([sys.executable, "-c", "from cgnn_amd import native; print(native.rt().__file__)"],
                           cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           timeout=300)
    assert probe.returncode == 0, probe.stderr[-3000:]
    assert os.path.samefile(probe.stdout.strip().splitlines()[-1], target)     # the sanitized build is in use
    res = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                          "tests/test_reorder_cpu.py", "tests/test_runtime_gnn_cpu.py"],
                         cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         timeout=1200)
    out = res.stdout
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert res.returncode == 0, out[-4000:]
    assert " passed" in out
