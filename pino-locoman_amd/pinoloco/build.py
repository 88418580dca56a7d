"""Build the HIP extension (libpinoloco.so) in-tree for gfx950.

The shared library is the product: every hot-path kernel plus the C-ABI of
``include/pinoloco.h``.  It is built next to this file so it travels with the
repository snapshot to the GPU box (``pino-locoman_amd/pinoloco/libpinoloco.so``).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.normpath(os.path.join(HERE, "..", "csrc"))
LIB = os.path.join(HERE, "libpinoloco.so")
SOURCES = ["api.hip", "api_build.hip", "api_casadi.hip", "k_eval.hip", "k_qp.hip", "k_admm.hip", "k_factor.hip", "k_dyn.hip", "k_admm2.hip", "k_ip.hip", "k_admm_rc.hip", "k_hess.hip"]
ARCH = os.environ.get("PL_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def _flags():
    # PL_HIPCC_DEFS: extra -D options for kernel A/B experiments (e.g. -DPL_JAC_WAVES=2)
    return ["-std=c++17", "-O3", f"--offload-arch={ARCH}", "-fPIC", "-Wno-unused-result", "-Wno-unused-value",
            "-I", CSRC, "-I", os.path.join(CSRC, "..", "..", "include")] + os.environ.get("PL_HIPCC_DEFS", "").split()


# Per-source code-generation options.  The ADMM sweeps run one or two waves per SIMD (no
# other wave hides their latency): the iterative ILP scheduler cuts k_admm 25.0 -> 24.5 ms
# per launch at the headline config and k_admm2 14.2 -> 13.8 ms at config 3
# (tools/gpu_libs.sh, tools/gpu_libs2.sh, profiles/r02f/sched/); it slows k_factor and
# k_eval_jac<0>, so it is not global.
_ILP = ["-mllvm", "--amdgpu-sched-strategy=iterative-ilp"]
SOURCE_FLAGS = {"k_admm.hip": _ILP, "k_admm2.hip": _ILP}
# PL_ILP_SOURCES: more sources to build with that scheduler (comma list, A/B experiments)
for _src in filter(None, os.environ.get("PL_ILP_SOURCES", "").split(",")):
    SOURCE_FLAGS[_src] = _ILP


INCLUDE = os.path.normpath(os.path.join(CSRC, "..", "..", "include"))


def source_sha() -> str:
    """sha256 over the library's sources: every file of csrc/ and include/ (name and bytes, in
    sorted order) plus this build script.  It is compiled into the library
    (``pl_build_info``), and ``build()`` rebuilds whenever the library on disk carries another
    hash -- file times are not trusted (a pushed tree keeps the builder's mtimes)."""
    h = hashlib.sha256()
    files = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))]
    files += [os.path.join(INCLUDE, f) for f in sorted(os.listdir(INCLUDE)) if f.endswith(".h")]
    files.append(os.path.abspath(__file__))
    for path in files:
        if not os.path.isfile(path):
            continue
        h.update(os.path.relpath(path, os.path.join(CSRC, "..", "..")).encode())
        h.update(b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    # the compile options, without the tree's absolute include paths (the GPU box runs the same
    # tree under another root)
    h.update(" ".join(f for f in _flags() if not os.path.isabs(f)).encode())
    return h.hexdigest()


def embedded_sha(path: str = LIB):
    """The source hash compiled into a built library (its pl_build_info string), or None."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    k = data.find(b"pl_src_sha256=")
    if k < 0:
        return None
    return data[k + 14:k + 14 + 64].decode("ascii", "replace")


def build(force: bool = False, verbose: bool = True) -> str:
    sha = source_sha()
    if not force and embedded_sha() == sha:
        return LIB
    hipcc = _hipcc()
    objdir = os.path.join(HERE, "_build")
    os.makedirs(objdir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(objdir, src.replace(".hip", ".o"))
        cmd = [hipcc] + _flags() + SOURCE_FLAGS.get(src, []) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if src == "api.hip":
            cmd.append(f'-DPL_SRC_SHA="{sha}"')
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-4000:]}")
        return obj

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"[pinoloco] built {LIB} (sources sha256 {sha[:16]})", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
