"""In-tree build of the native extension ``ops/_C*.so`` for gfx950.

No hipify, no ``torch.utils.cpp_extension.CUDAExtension`` (which would
run hipify over the sources): the HIP kernels are compiled directly with
``hipcc --offload-arch=gfx950`` and the pybind/torch binding with the host
compiler, then linked against PyTorch-ROCm's own HIP runtime
(``torch/lib/libamdhip64.so``, SONAME ``libamdhip64.so.7``) so the process
has exactly one HIP runtime.

Usage: ``python -m pytorch_distributed_matmul_benchmark_amd.ops.build``
(or ``build()`` from Python). Rebuilds only when a source is newer than
the library.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE / "_build"
ARCH = os.environ.get("PDMB_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_C"

HIP_SOURCES = ["gemm_mfma256.hip", "gemm_f32_256.hip", "gemm_fp8.hip", "gemm_generic.hip", "gemm_w4.hip",
               "gemm_tile.hip", "gemm_f32_w4.hip", "gemm_f32_tile.hip", "reduce.hip", "gemm_dispatch.cpp"]
HOST_SOURCES = ["bindings.cpp"]


def rocm_path() -> Path:
    return Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def hipcc() -> str:
    p = rocm_path() / "bin" / "hipcc"
    return str(p) if p.exists() else (shutil.which("hipcc") or "hipcc")


def lib_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return HERE / f"{EXT_NAME}{suffix}"


def _torch_paths():
    import torch  # noqa: F401
    from torch.utils import cpp_extension

    return cpp_extension.include_paths(), cpp_extension.library_paths()


def _needs_build(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def experiments() -> bool:
    """``PDMB_EXPERIMENTS=1``: also compile the A/B and timing-only diagnostic
    kernels (api.h ``ExperimentKernel``). The default build ships without them."""
    return os.environ.get("PDMB_EXPERIMENTS", "0") == "1"


def source_files():
    return ([CSRC / s for s in HIP_SOURCES + HOST_SOURCES] + sorted(CSRC.glob("*.h"))
            + [Path(__file__)])


def source_digest() -> str:
    """Content hash of every source the extension is built from plus the build
    flags. Stored next to the library (``stamp_path``) at build time and
    compared by ``_native.load`` — content, not mtimes, so a copied tree
    (gpurun snapshot, git checkout) is judged correctly."""
    import hashlib

    h = hashlib.sha256()
    for p in source_files():
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(f"arch={ARCH};experiments={int(experiments())}".encode())
    return h.hexdigest()


def stamp_path() -> Path:
    return HERE / f"{EXT_NAME}.sources.sha256"


def is_stale() -> bool:
    """True if the built library is missing or was built from other sources / flags."""
    if not lib_path().exists() or not stamp_path().exists():
        return True
    return stamp_path().read_text().strip() != source_digest()


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}): {' '.join(map(str, cmd))}\n"
                           f"{r.stdout}\n{r.stderr}")
    return r


RUNTIME = HERE.parent / "runtime"
BENCH_SRC = RUNTIME / "pdmb_bench.cpp"


def bench_path() -> Path:
    return RUNTIME / "pdmb_bench"


def build_bench(verbose: bool = False, force: bool = False) -> Path:
    """Link the Python-free native executor ``runtime/pdmb_bench`` (HIP + RCCL) from
    ``runtime/pdmb_bench.cpp`` and the same kernel objects as ``_C``."""
    build(verbose=verbose, force=force)  # kernel objects
    out = bench_path()
    objs = [BUILD / (Path(s).stem + ".o") for s in HIP_SOURCES]
    deps = [BENCH_SRC, CSRC / "api.h"] + objs
    if not force and not _needs_build(out, deps):
        return out
    rocm = rocm_path()
    obj = BUILD / "pdmb_bench.o"
    # compile and link separately: hipcc's implicit "-x hip" would otherwise
    # also apply to the kernel objects on the link line
    _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", f"-I{CSRC}",
          f"-I{rocm / 'include'}", "-c", BENCH_SRC, "-o", obj], verbose)
    _run([hipcc(), f"--offload-arch={ARCH}", obj, *objs, "-o", out, f"-L{rocm / 'lib'}", "-lrccl",
          "-lpthread", f"-Wl,-rpath,{rocm / 'lib'}"], verbose)
    return out


PROBE_SRC = RUNTIME / "mfma_probe.hip"


def probe_path() -> Path:
    return RUNTIME / "mfma_probe"


def build_probe(verbose: bool = False, force: bool = False) -> Path:
    """The stand-alone MFMA-shape probe (runtime/mfma_probe.hip): 16x16x32 vs
    32x32x16 bf16 FLOP rate on random operands (profiles/r2_mfma_shape_probe.jsonl)."""
    out = probe_path()
    if force or _needs_build(out, [PROBE_SRC]):
        _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", PROBE_SRC, "-o", out], verbose)
    return out


MASK_PROBE_SRC = RUNTIME / "cu_mask_probe.hip"


def build_mask_probe(verbose: bool = False, force: bool = False) -> Path:
    """The stand-alone CU-mask placement probe (runtime/cu_mask_probe.hip): which
    XCD / CU each workgroup of a CU-masked stream runs on."""
    out = RUNTIME / "cu_mask_probe"
    if force or _needs_build(out, [MASK_PROBE_SRC]):
        _run([hipcc(), f"--offload-arch={ARCH}", "-O2", "-std=c++17", MASK_PROBE_SRC, "-o", out], verbose)
    return out


def build(verbose: bool = False, force: bool = False, jobs: int | None = None) -> Path:
    """Compile every HIP/C++ source for gfx950 and link ``_C``. Returns the .so path."""
    headers = sorted(CSRC.glob("*.h"))
    out = lib_path()
    digest = source_digest()
    if not force and not is_stale():
        return out
    BUILD.mkdir(exist_ok=True)
    # a flag change (PDMB_EXPERIMENTS) invalidates every object
    flags_file = BUILD / "flags.txt"
    flags = f"arch={ARCH};experiments={int(experiments())}"
    if not flags_file.exists() or flags_file.read_text() != flags:
        force = True
    # Until this build links, the objects may be a mix of flavours (a failed
    # PDMB_EXPERIMENTS=1 build leaves its objects behind, newer than their
    # sources): with no flags file, the next build of either flavour starts over.
    flags_file.unlink(missing_ok=True)
    inc, libdirs = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    import torch

    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    hip_flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                 "-Wno-unused-result", "-munsafe-fp-atomics", f"-I{CSRC}"]
    if experiments():
        hip_flags.append("-DPDMB_EXPERIMENTS=1")
    host_flags = ["-O2", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                  f"-DTORCH_EXTENSION_NAME={EXT_NAME}", "-DTORCH_API_INCLUDE_EXTENSION_H",
                  "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-I{CSRC}",
                  f"-I{rocm_path() / 'include'}", f"-I{py_inc}"] + [f"-I{p}" for p in inc]

    steps = []
    objs = []
    for s in HIP_SOURCES:
        src = CSRC / s
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _needs_build(obj, [src] + headers):
            lang = ["-x", "hip"] if src.suffix == ".cpp" else []
            steps.append([hipcc()] + hip_flags + lang + ["-c", src, "-o", obj])
    cxx = os.environ.get("CXX", "g++")
    for s in HOST_SOURCES:
        src = CSRC / s
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _needs_build(obj, [src] + headers):
            steps.append([cxx] + host_flags + ["-c", src, "-o", obj])

    jobs = jobs or min(len(steps) or 1, max(1, (os.cpu_count() or 2) // 2), 8)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), steps))

    torch_lib = libdirs[0]
    link = [cxx, "-shared", "-o", out] + objs + [
        f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
        "-ltorch_python", "-lamdhip64", f"-Wl,-rpath,{torch_lib}"]
    _run(link, verbose)
    flags_file.write_text(flags)
    stamp_path().write_text(digest + "\n")
    return out


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--no-bench", action="store_true", help="skip the native pdmb_bench executable")
    a = ap.parse_args(argv)
    p = build(verbose=a.verbose, force=a.force)
    print(p)
    if not a.no_bench:
        print(build_bench(verbose=a.verbose))
        print(build_probe(verbose=a.verbose))
        print(build_mask_probe(verbose=a.verbose))


if __name__ == "__main__":
    sys.exit(main())
