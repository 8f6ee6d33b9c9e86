#!/usr/bin/env python3
"""Build the native extensions of jax_llama_amd IN-TREE (gfx950 only).

  * ``jax_llama_amd/_C*.so``   — the HIP kernels (``csrc/kernels/*.hip``, hipcc
    ``--offload-arch=gfx950``) + torch bindings (``csrc/bindings.cpp``);
  * ``jax_llama_amd/_bpe*.so`` — the C++ byte-pair-merge core of the Llama-3 tokenizer.

The xGMI custom all-reduce (``csrc/kernels/allreduce.hip``) is part of ``_C``.

No hipify, no CUDA, no JIT cache: objects go to ``build/`` (incremental, mtime based) and the
final ``.so`` files land next to the Python package so they travel with the repo snapshot.

Usage: ``python build.py [-j N] [--force] [--only C|bpe] [--debug-bounds]``

``--debug-bounds`` additionally builds ``jax_llama_amd/_C_dbg*.so`` (objects in ``build/C_dbg``) with
``-DJLA_DEBUG_BOUNDS``: every clamped / skipped out-of-range index that comes from device state (token ids,
the KV-cache slot, RoPE positions, the sequence length) sets a bit in an error word the host can read
(``ops.bounds_error()``). ``JLA_DEBUG_BOUNDS=1`` makes ``ops.ext()`` load it instead of ``_C``.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "jax_llama_amd"
CSRC = PKG / "csrc"
BUILD = ROOT / "build"
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX")


def _torch_paths():
    import torch
    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    return tdir, inc, tdir / "lib"


def _py_include():
    return sysconfig.get_paths()["include"]


def _pybind_include():
    import pybind11
    return pybind11.get_include()


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(map(str, cmd)) + "\n" + r.stdout)
        raise SystemExit(f"build failed: {cmd[-1]}")
    return r.stdout


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-D__HIP_PLATFORM_AMD__"]


def _scratch_users(remarks: str):
    """Kernels whose resource-usage remark reports scratch (private) memory: on these kernels that
    means a runtime-indexed register array or a spill -- almost always a large slowdown."""
    bad, name = [], None
    for line in remarks.splitlines():
        if "Function Name:" in line:
            name = line.split("Function Name:")[1].split("[")[0].strip()
        elif "ScratchSize [bytes/lane]:" in line and name:
            size = int(line.split("ScratchSize [bytes/lane]:")[1].split("[")[0].strip())
            if size > 0:
                bad.append((name, size))
    return bad


# Kernels allowed to use scratch, by mangled-name substring -> max bytes/lane (a rare shape where a spill is accepted).
# Empty: no kernel of the release or the bounds-checked build spills (re-checked in round 6 after the stream-K, fixup
# and exchange-split plans whose epilogue spills these entries used to allow were deleted).
SCRATCH_OK: dict = {}


def _compile_hip(src: Path, obj: Path, headers, force: bool, extra=()):
    if force or _stale(obj, [src, *headers]):
        obj.parent.mkdir(parents=True, exist_ok=True)
        out = _run([HIPCC, *HIP_FLAGS, *extra, "-Rpass-analysis=kernel-resource-usage", "-c", str(src), "-o",
                    str(obj)])
        bad = [(n, b) for n, b in _scratch_users(out) if not any(ok in n and b <= lim for ok, lim in SCRATCH_OK.items())]
        if bad:
            obj.unlink(missing_ok=True)
            raise SystemExit(f"{src.name}: kernels use scratch memory (runtime-indexed register array or spill): "
                             + ", ".join(f"{n} ({b} B/lane)" for n, b in bad))
        return True
    return False


def build_C(jobs: int, force: bool, debug_bounds: bool = False) -> Path:
    tdir, tinc, tlib = _torch_paths()
    kdir = CSRC / "kernels"
    headers = sorted(kdir.glob("*.h"))
    srcs = sorted(kdir.glob("*.hip"))
    name = "_C_dbg" if debug_bounds else "_C"
    odir = BUILD / ("C_dbg" if debug_bounds else "C")
    extra = ["-DJLA_DEBUG_BOUNDS"] if debug_bounds else []
    objs = [odir / (s.stem + ".o") for s in srcs]
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        rebuilt = list(ex.map(lambda so: _compile_hip(so[0], so[1], headers, force, extra), zip(srcs, objs)))
    # the hand-counted load rings must never be read before their waits: check the assembly
    for src, did in zip(srcs, rebuilt):
        if did and src.stem in ("gemv", "attn_decode", "attn_decode_mma"):  # (attn_decode: the v4 ring)
            asm = odir / (src.stem + ".s")
            _run([HIPCC, *HIP_FLAGS, *extra, "--cuda-device-only", "-S", str(src), "-o", str(asm)])
            try:
                _run([sys.executable, str(ROOT / "tools" / "check_asm_ring.py"), str(asm)])
            except SystemExit:
                # the object must not survive a failed check: it would look up to date to the next build
                (odir / (src.stem + ".o")).unlink(missing_ok=True)
                raise
    bsrc = CSRC / "bindings.cpp"
    bobj = odir / "bindings.o"
    if force or _stale(bobj, [bsrc, *headers]):
        inc = [f"-I{p}" for p in tinc] + [f"-I{_py_include()}", f"-I{CSRC}"]
        # host code only (no kernels in the bindings): skip the device pass
        _run([HIPCC, "-O2", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "--offload-host-only",
              "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
              f"-DTORCH_EXTENSION_NAME={name}", *extra, "-DTORCH_API_INCLUDE_EXTENSION_H", "-D_GLIBCXX_USE_CXX11_ABI=1",
              "-Wno-deprecated-declarations", "-Wno-unused-result", *inc, "-c", str(bsrc), "-o", str(bobj)])
    out = PKG / f"{name}{EXT_SUFFIX}"
    if force or _stale(out, [*objs, bobj]):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), str(bobj), "-o", str(out),
              f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
              "-lamdhip64", f"-Wl,-rpath,{tlib}"])
    return out


def build_bpe(force: bool) -> Path:
    src = CSRC / "bpe" / "bpe.cpp"
    out = PKG / f"_bpe{EXT_SUFFIX}"
    if force or _stale(out, [src]):
        _run(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", f"-I{_pybind_include()}", f"-I{_py_include()}",
              str(src), "-o", str(out)])
    return out


def build_all(jobs: int = 8, force: bool = False, only=None, debug_bounds: bool = False):
    outs = []
    if only in (None, "bpe"):
        outs.append(build_bpe(force))
    if only in (None, "C"):
        outs.append(build_C(jobs, force))
        if debug_bounds:
            outs.append(build_C(jobs, force, debug_bounds=True))
    return outs


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["C", "bpe"])
    ap.add_argument("--debug-bounds", action="store_true", help="also build the bounds-checked _C_dbg extension")
    a = ap.parse_args()
    for o in build_all(a.j, a.force, a.only, a.debug_bounds):
        print("built", o.relative_to(ROOT))
