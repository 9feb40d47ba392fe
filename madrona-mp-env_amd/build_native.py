"""Builds the native parts of the engine in-tree (no JIT cache, no pip).

Outputs (git-ignored, shipped to the GPU box with the snapshot):
  madrona-mp-env_amd/libmpenv.so                     HIP kernels + C ABI (gfx950)
  madrona-mp-env_amd/madrona_mp_env<ext-suffix>.so   Python module (pybind11)
  oracle/_build/liboracle.so                         CPU parity oracle (tests only)

Every float translation unit is compiled with -ffp-contract=off so the host
oracle and the gfx950 kernels round identically (see csrc/mpenv_core.h).
"""
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
ORACLE = os.path.join(ROOT, "oracle")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MPENV_OFFLOAD_ARCH", "gfx950")

LIB = os.path.join(PKG, "libmpenv.so")
EXT = os.path.join(PKG, "madrona_mp_env" + sysconfig.get_config_var("EXT_SUFFIX"))
ORACLE_LIB = os.path.join(ORACLE, "_build", "liboracle.so")

LIB_SOURCES = ["kernels.hip", "wire.hip", "manager.cpp", "scene.cpp", "navmesh.cpp"]
LIB_HEADERS = ["mpenv_core.h", "engine.h", "geom_dev.h", "scene.h"]


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    # stderr: callers such as bench.py own stdout (one JSON line)
    print("[build]", " ".join(cmd), file=sys.stderr, flush=True)
    subprocess.run(cmd, check=True, stdout=sys.stderr)


def build_lib(force=False):
    srcs = [os.path.join(CSRC, s) for s in LIB_SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in LIB_HEADERS] + [os.path.join(INCLUDE, "mpenv.h")]
    if not force and not _stale(LIB, deps):
        return LIB
    objdir = os.path.join(PKG, "build")
    os.makedirs(objdir, exist_ok=True)
    objs = []
    common = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
              f"-I{CSRC}", f"-I{INCLUDE}", "-Wall", "-Wno-unused-variable",
              "-Wno-unused-function"]
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        if s.endswith(".hip"):
            cmd = [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-c", s, "-o", o] + common
        else:
            cmd = [HIPCC, "-x", "c++", "-c", s, "-o", o] + common + ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        _run(cmd)
        objs.append(o)
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs +
         ["-Wl,-soname,libmpenv.so"])
    return LIB


def build_ext(force=False):
    src = os.path.join(CSRC, "pybind_module.cpp")
    if not os.path.exists(src):
        return None
    if not force and not _stale(EXT, [src, LIB, os.path.join(INCLUDE, "mpenv.h")]):
        return EXT
    import pybind11
    py_inc = sysconfig.get_paths()["include"]
    _run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", f"-I{pybind11.get_include()}",
          f"-I{py_inc}", f"-I{INCLUDE}", src, "-o", EXT, f"-L{PKG}", "-lmpenv",
          "-Wl,-rpath,$ORIGIN"])
    return EXT


HEADLESS = os.path.join(PKG, "headless")


def build_headless(force=False):
    """C++ driver over include/mpenv_manager.hpp (reference src/headless.cpp role)."""
    src = os.path.join(CSRC, "headless.cpp")
    deps = [src, LIB, os.path.join(INCLUDE, "mpenv.h"), os.path.join(INCLUDE, "mpenv_manager.hpp"),
            os.path.join(CSRC, "mpenv_core.h")]
    if not force and not _stale(HEADLESS, deps):
        return HEADLESS
    _run([HIPCC, "-x", "c++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
          f"-I{INCLUDE}", f"-I{CSRC}", src, "-o", HEADLESS, f"-L{PKG}", "-lmpenv",
          "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"])
    return HEADLESS


def build_oracle(force=False):
    src = os.path.join(ORACLE, "oracle.cpp")
    deps = [src, os.path.join(ORACLE, "oracle.h"), os.path.join(CSRC, "mpenv_core.h"),
            os.path.join(INCLUDE, "mpenv.h")]
    if not force and not _stale(ORACLE_LIB, deps):
        return ORACLE_LIB
    os.makedirs(os.path.dirname(ORACLE_LIB), exist_ok=True)
    _run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
          "-Wall", "-Wno-invalid-offsetof", f"-I{INCLUDE}", f"-I{CSRC}", src, "-o", ORACLE_LIB,
          "-lpthread"])
    return ORACLE_LIB


def build_all(force=True):
    """Every artefact, recompiled from source by default (build() must never
    ship binaries it did not compile); force=False is the incremental mode
    the test harness uses when a build already ran in this tree."""
    build_lib(force)
    build_ext(force)
    build_headless(force)
    build_oracle(force)


if __name__ == "__main__":
    build_all(force="--incremental" not in sys.argv)
