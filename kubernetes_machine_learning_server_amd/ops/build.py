"""In-tree build of the native extension ``_native`` (C++17 host runtime + gfx950 HIP kernels).

Every translation unit is compiled by ``hipcc`` (``.hip`` with ``--offload-arch=gfx950``,
``.cpp`` as plain host C++), then linked into
``kubernetes_machine_learning_server_amd/_native<EXT_SUFFIX>``.  No torch cpp_extension, no
hipify: the sources are HIP already.  Incremental: an object is rebuilt when its source or any
header is newer.  ``python -m kubernetes_machine_learning_server_amd.ops.build [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import pathlib
import shutil
import subprocess
import sys
import sysconfig
from typing import List

ROOT = pathlib.Path(__file__).resolve().parents[2]
PKG = ROOT / "kubernetes_machine_learning_server_amd"
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
ARCH = os.environ.get("KMLS_OFFLOAD_ARCH", "gfx950")


def ext_path() -> pathlib.Path:
    return PKG / ("_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build kmls native code)")


def sources() -> List[pathlib.Path]:
    out = sorted((CSRC / "host").glob("*.cpp")) + sorted((CSRC / "host").glob("*.hip"))
    out += sorted((CSRC / "kernels").glob("*.hip"))
    return out


def _headers() -> List[pathlib.Path]:
    return list(CSRC.rglob("*.hpp")) + list(CSRC.rglob("*.h"))


def _includes() -> List[str]:
    import pybind11
    return [f"-I{CSRC / 'include'}", f"-I{pybind11.get_include()}",
            f"-I{sysconfig.get_paths()['include']}"]


def _obj_for(src: pathlib.Path) -> pathlib.Path:
    rel = src.relative_to(CSRC)
    return BUILD / (str(rel).replace(os.sep, "__") + ".o")


def _compile(src: pathlib.Path, force: bool, hdr_mtime: float) -> str:
    obj = _obj_for(src)
    if (not force and obj.exists() and obj.stat().st_mtime >= src.stat().st_mtime
            and obj.stat().st_mtime >= hdr_mtime):
        return f"[up-to-date] {src.name}"
    cmd = [_hipcc(), "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result",
           "-fvisibility=hidden", "-march=x86-64-v2"] + _includes()
    if src.suffix == ".hip":
        cmd += ["-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
    cmd += ["-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return f"[built] {src.name}"


def build(force: bool = False, jobs: int = 0, verbose: bool = False) -> pathlib.Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    hdr_mtime = max((h.stat().st_mtime for h in _headers()), default=0.0)
    jobs = jobs or min(8, os.cpu_count() or 4, int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for msg in ex.map(lambda s: _compile(s, force, hdr_mtime), srcs):
            if verbose:
                print(msg, flush=True)
    out = ext_path()
    objs = [_obj_for(s) for s in srcs]
    newest = max(o.stat().st_mtime for o in objs)
    if force or not out.exists() or out.stat().st_mtime < newest:
        tmp = out.with_suffix(".tmp.so")
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp)] + \
              [str(o) for o in objs] + ["-lpthread"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
        os.replace(tmp, out)
        if verbose:
            print(f"[linked] {out}", flush=True)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    a = ap.parse_args(argv)
    print(build(a.force, a.jobs, verbose=True))
    return 0


if __name__ == "__main__":
    sys.exit(main())
