"""In-tree build of the native extensions (no JIT cache, no hipify).

* ``cgnn_amd/_hip*.so``  -- HIP kernels + pybind11 bindings, ``hipcc --offload-arch=gfx950``
* ``cgnn_amd/_rt*.so``   -- host C++ runtime (DAG-program compiler, graph
                            algorithms, CSR builder, synthetic graph generator,
                            neighbour sampler), plain ``g++ -O3 -fopenmp``

Usage: ``python -m cgnn_amd._build [--force] [--only hip|rt] [--debug]``.
A rebuild happens only when a source is newer than the target.
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("CGNN_OFFLOAD_ARCH", "gfx950")


def _pybind_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _newer(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout)
        raise RuntimeError("native build failed: %s" % cmd[0])
    if verbose and res.stdout.strip():
        print(res.stdout)


def hip_target():
    return os.path.join(HERE, "_hip" + EXT)


def rt_target():
    return os.path.join(HERE, "_rt" + EXT)


def build_hip(force=False, verbose=False, debug=False):
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    srcs += sorted(glob.glob(os.path.join(CSRC, "kernels", "*.cpp")))
    hdrs = glob.glob(os.path.join(CSRC, "include", "*.h"))
    target = hip_target()
    if not force and not _newer(target, srcs + hdrs + [__file__]):
        return target
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    inc = ["-I" + os.path.join(CSRC, "include")] + ["-I" + p for p in _pybind_includes()]
    opt = ["-O0", "-g"] if debug else ["-O3"]
    objdir = os.path.join(HERE, "..", "build", "hip")
    os.makedirs(objdir, exist_ok=True)
    objs, cmds = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs + [__file__]):
            lang = ["-x", "hip", "--offload-arch=" + ARCH] if s.endswith(".hip") else []
            cmds.append([hipcc, "-c", "-fPIC", "-std=c++17", *opt, *lang, *inc,
                         "-Wno-unused-result", "-fvisibility=hidden", s, "-o", o])
    # one hipcc per translation unit, a few at a time (each holds 1-3 GB while it
    # optimises the larger kernel files)
    jobs = max(1, min(len(cmds), int(os.environ.get("CGNN_BUILD_JOBS", "4"))))
    if jobs > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(jobs) as pool:
            list(pool.map(lambda c: _run(c, verbose), cmds))
    else:
        for c in cmds:
            _run(c, verbose)
    cmd = [hipcc, "-shared", "-fPIC", "--offload-arch=" + ARCH, *objs, "-o", target]
    _run(cmd, verbose)
    return target


def build_rt(force=False, verbose=False, debug=False, target=None):
    """Host C++ runtime module ``_rt``.  ``debug``: -O1 -g with AddressSanitizer and
    UndefinedBehaviorSanitizer (errors abort; load it with ``CGNN_RT_LIB=<target>`` and
    ``LD_PRELOAD`` of the compiler's libasan -- ``tests/test_sanitizers_cpu.py``)."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    target = target or rt_target()
    if not srcs:
        return None
    if not force and not _newer(target, srcs + hdrs + [__file__]):
        return target
    cxx = os.environ.get("CXX", "g++")
    inc = ["-I" + os.path.join(CSRC, "runtime")] + ["-I" + p for p in _pybind_includes()]
    opt = (["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
            "-fno-sanitize-recover=undefined"] if debug else ["-O3"])
    cmd = [cxx, "-shared", "-fPIC", "-std=c++17", *opt, "-fopenmp", "-fvisibility=hidden",
           *inc, *srcs, "-o", target]
    _run(cmd, verbose)
    return target


def build_all(force=False, verbose=False, debug=False):
    return build_rt(force, verbose, debug), build_hip(force, verbose, debug)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["hip", "rt"])
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    if a.only in (None, "rt"):
        print(build_rt(a.force, a.verbose, a.debug))
    if a.only in (None, "hip"):
        print(build_hip(a.force, a.verbose, a.debug))
