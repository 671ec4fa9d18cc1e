"""In-tree native build of the framework (no setup.py / JIT cache).

Products (all git-ignored, shipped to GPU boxes with the repo snapshot):
  boinc_app_eah_brp_amd/_brp<EXT_SUFFIX>   Python extension (pybind11)
  bin/einsteinbinary_mi355x                BOINC application (C++ main)
  build/obj/*.o                            object cache
  --checked: boinc_app_eah_brp_amd/_brp_checked<EXT_SUFFIX> and
  bin/einsteinbinary_mi355x_checked, the device-side debug build
  (csrc/hip/checked.hpp: serialised, verified launches and bounds-checked
  kernel accesses; BRP_CHECKED=1 makes the package load it)

Device code is compiled for gfx950 only with hipcc; host-only C++ with
amdclang++. Run:  python -m boinc_app_eah_brp_amd._build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
PKG = ROOT / "boinc_app_eah_brp_amd"
BIN = ROOT / "bin"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")
CLANG = str(ROCM / "llvm" / "bin" / "clang++")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]

HOST_SRCS = [
    "core/log.cpp", "core/io.cpp", "core/stats.cpp", "core/gsl_compat.cpp", "core/rngmed.cpp",
    "core/search_core.cpp", "core/cpu_fft.cpp", "core/cpu_backend.cpp", "core/wisdom.cpp", "core/trace.cpp",
    "boinc/runtime.cpp", "boinc/crash.cpp", "boinc/ipc.cpp",
    "engine/cpu_engine.cpp", "engine/hip_engine.cpp", "engine/checked.cpp",
    "app/search.cpp", "app/multi.cpp", "app/passes.cpp", "app/cli.cpp",
]
DEVICE_SRCS = [
    "hip/fft_passes.hip", "hip/bluestein.hip", "hip/harmonic_sum.hip", "hip/resample.hip", "hip/whiten.hip", "hip/rmed_wide.hip",
    "hip/checked.hip",
]
BINDING_SRCS = ["bindings/pybind.cpp"]
APP_MAIN = "app/main.cpp"


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def extension_path() -> Path:
    return PKG / f"_brp{ext_suffix()}"


def app_path() -> Path:
    return BIN / "einsteinbinary_mi355x"


def git_id() -> str:
    try:
        return subprocess.check_output(["git", "-C", str(ROOT), "rev-parse", "HEAD"], stderr=subprocess.DEVNULL,
                                       text=True).strip()
    except Exception:
        return "unknown"


def _common_flags() -> list[str]:
    return ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-Wno-unknown-pragmas",
            "-D__HIP_PLATFORM_AMD__", f"-I{ROCM / 'include'}", f'-DBRP_GIT_ID="{git_id()[:40]}"',
            *os.environ.get("BRP_EXTRA_CFLAGS", "").split()]  # experiment builds (scripts/build_variant.sh)


def _headers_mtime() -> float:
    return max(p.stat().st_mtime for p in CSRC.rglob("*.hpp"))


def _needs(obj: Path, src: Path, hdr_mtime: float, force: bool) -> bool:
    if force or not obj.exists():
        return True
    return obj.stat().st_mtime < max(src.stat().st_mtime, hdr_mtime)


# Host-code sanitizers: the app is also built with ASan +
# UBSan on every host translation unit (device code is not instrumented: GPU
# sanitizers are not available on the MI355X pool). On hipcc lines each
# -fsanitize= follows -Xarch_host so only the host compilation sees it.
SAN = ["address", "undefined"]
OBJ_SAN = ROOT / "build" / "obj_asan"


def asan_app_path() -> Path:
    return BIN / "einsteinbinary_mi355x_asan"


OBJ_CHECKED = ROOT / "build" / "obj_checked"


def checked_extension_path() -> Path:
    return PKG / f"_brp_checked{ext_suffix()}"


def checked_app_path() -> Path:
    return BIN / "einsteinbinary_mi355x_checked"


def _compile(src_rel: str, force: bool, hdr_mtime: float, sanitize: bool = False,
             checked: bool = False) -> tuple[str, Path]:
    src = CSRC / src_rel
    obj = (OBJ_SAN if sanitize else OBJ_CHECKED if checked else OBJ) / (src_rel.replace("/", "__") + ".o")
    if not _needs(obj, src, hdr_mtime, force):
        return "cached", obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    san_host = [f for s in SAN for f in ("-Xarch_host", f"-fsanitize={s}")] if sanitize else []
    san_cxx = [f"-fsanitize={s}" for s in SAN] + ["-fno-omit-frame-pointer", "-g"] if sanitize else []
    chk = ["-DBRP_CHECKED=1"] if checked else []
    if src.suffix == ".hip":
        cmd = [HIPCC, f"--offload-arch={ARCH}", *_common_flags(), *chk, "-munsafe-fp-atomics", *san_host,
               *(["-Xarch_host", "-fno-omit-frame-pointer"] if sanitize else []), "-c", str(src), "-o", str(obj)]
    else:
        flags = _common_flags() + chk + san_cxx
        if src_rel.startswith("bindings/"):
            import pybind11
            flags += [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
                      "-fvisibility=hidden"]
            if checked:
                flags += ["-DBRP_MODULE_NAME=_brp_checked"]
        cmd = [CLANG, *flags, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src_rel}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return "built", obj


def _link(objs: list[Path], out: Path, shared: bool, sanitize: bool = False) -> None:
    out.parent.mkdir(parents=True, exist_ok=True)
    tmp = out.with_name(out.name + ".tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", *[str(o) for o in objs], "-o", str(tmp),
           f"-L{ROCM / 'lib'}", "-lamdhip64", "-lz", "-lpthread", "-ldl"]
    if sanitize:
        cmd += [f"-fsanitize={s}" for s in SAN]
    if shared:
        cmd.insert(1, "-shared")
    else:
        cmd += [f"-Wl,-rpath,{ROCM / 'lib'}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {out}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> dict:
    jobs = jobs or min(16, os.cpu_count() or 4)
    hdr = _headers_mtime()
    srcs = HOST_SRCS + DEVICE_SRCS + BINDING_SRCS + [APP_MAIN]
    results = {}
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(_compile, s, force, hdr): s for s in srcs}
        for f in cf.as_completed(futs):
            status, obj = f.result()
            results[futs[f]] = obj
            if verbose and status == "built":
                print(f"[build] {futs[f]}", flush=True)
    core = [results[s] for s in HOST_SRCS + DEVICE_SRCS]
    ext = extension_path()
    ext_objs = core + [results[s] for s in BINDING_SRCS]
    if force or not ext.exists() or ext.stat().st_mtime < max(o.stat().st_mtime for o in ext_objs):
        _link(ext_objs, ext, shared=True)
        if verbose:
            print(f"[build] linked {ext.relative_to(ROOT)}", flush=True)
    app = app_path()
    app_objs = core + [results[APP_MAIN]]
    if force or not app.exists() or app.stat().st_mtime < max(o.stat().st_mtime for o in app_objs):
        _link(app_objs, app, shared=False)
        if verbose:
            print(f"[build] linked {app.relative_to(ROOT)}", flush=True)
    return {"extension": str(ext), "app": str(app)}


def build_asan(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    """ASan + UBSan build of the application binary (host code instrumented)."""
    jobs = jobs or min(16, os.cpu_count() or 4)
    hdr = _headers_mtime()
    srcs = HOST_SRCS + DEVICE_SRCS + [APP_MAIN]
    results = {}
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(_compile, s, force, hdr, True): s for s in srcs}
        for f in cf.as_completed(futs):
            status, obj = f.result()
            results[futs[f]] = obj
            if verbose and status == "built":
                print(f"[build asan] {futs[f]}", flush=True)
    objs = [results[s] for s in srcs]
    app = asan_app_path()
    if force or not app.exists() or app.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        _link(objs, app, shared=False, sanitize=True)
        if verbose:
            print(f"[build asan] linked {app.relative_to(ROOT)}", flush=True)
    return app


OBJ_TSAN = ROOT / "build" / "obj_tsan"


def tsan_app_path() -> Path:
    return BIN / "einsteinbinary_mi355x_tsan"


def build_tsan(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    """ThreadSanitizer build of the application (SURVEY.md 5.2 race detection):
    every host translation unit instrumented; the device modules' objects are
    the product build's (their host side is only kernel stubs and launchers,
    which the CPU backend never calls)."""
    jobs = jobs or min(16, os.cpu_count() or 4)
    hdr = _headers_mtime()
    prod = build(force=False, jobs=jobs, verbose=False)  # the device objects
    del prod
    srcs = HOST_SRCS + [APP_MAIN]

    def comp(src_rel: str) -> tuple[str, Path]:
        src = CSRC / src_rel
        obj = OBJ_TSAN / (src_rel.replace("/", "__") + ".o")
        if not _needs(obj, src, hdr, force):
            return "cached", obj
        obj.parent.mkdir(parents=True, exist_ok=True)
        flags = [f for f in _common_flags() if f != "-O3"] + ["-O1", "-g", "-fsanitize=thread", "-fno-omit-frame-pointer"]
        cmd = [CLANG, *flags, "-c", str(src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src_rel}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return "built", obj

    results = {}
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(comp, s): s for s in srcs}
        for f in cf.as_completed(futs):
            status, obj = f.result()
            results[futs[f]] = obj
            if verbose and status == "built":
                print(f"[build tsan] {futs[f]}", flush=True)
    objs = [results[s] for s in HOST_SRCS] + [OBJ / (s.replace("/", "__") + ".o") for s in DEVICE_SRCS]
    objs.append(results[APP_MAIN])
    app = tsan_app_path()
    if force or not app.exists() or app.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        out = app.with_name(app.name + ".tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", *[str(o) for o in objs], "-o", str(out), f"-L{ROCM / 'lib'}",
               "-lamdhip64", "-lz", "-lpthread", "-ldl", "-fsanitize=thread", f"-Wl,-rpath,{ROCM / 'lib'}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {app}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(out, app)
        if verbose:
            print(f"[build tsan] linked {app.relative_to(ROOT)}", flush=True)
    return app


def build_checked(force: bool = False, jobs: int | None = None, verbose: bool = True) -> dict:
    """Device-side debug build (csrc/hip/checked.hpp): module _brp_checked and
    bin/einsteinbinary_mi355x_checked."""
    jobs = jobs or min(16, os.cpu_count() or 4)
    hdr = _headers_mtime()
    srcs = HOST_SRCS + DEVICE_SRCS + BINDING_SRCS + [APP_MAIN]
    results = {}
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(_compile, s, force, hdr, False, True): s for s in srcs}
        for f in cf.as_completed(futs):
            status, obj = f.result()
            results[futs[f]] = obj
            if verbose and status == "built":
                print(f"[build checked] {futs[f]}", flush=True)
    core = [results[s] for s in HOST_SRCS + DEVICE_SRCS]
    ext = checked_extension_path()
    ext_objs = core + [results[s] for s in BINDING_SRCS]
    if force or not ext.exists() or ext.stat().st_mtime < max(o.stat().st_mtime for o in ext_objs):
        _link(ext_objs, ext, shared=True)
        if verbose:
            print(f"[build checked] linked {ext.relative_to(ROOT)}", flush=True)
    app = checked_app_path()
    app_objs = core + [results[APP_MAIN]]
    if force or not app.exists() or app.stat().st_mtime < max(o.stat().st_mtime for o in app_objs):
        _link(app_objs, app, shared=False)
        if verbose:
            print(f"[build checked] linked {app.relative_to(ROOT)}", flush=True)
    return {"checked_extension": str(ext), "checked_app": str(app)}


def build_with_checked(force: bool = False, jobs: int | None = None, verbose: bool = True) -> dict:
    """The product and the checked build side by side (two compile pools): each
    is dominated by its own fft_passes.hip, so a fresh tree builds in about the
    time of one."""
    with cf.ThreadPoolExecutor(max_workers=2) as ex:
        prod = ex.submit(build, force, jobs, verbose)
        chk = ex.submit(build_checked, force, jobs, verbose)
        out = prod.result()
        out.update(chk.result())
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--asan", action="store_true", help="also build bin/einsteinbinary_mi355x_asan (ASan + UBSan)")
    ap.add_argument("--tsan", action="store_true", help="also build bin/einsteinbinary_mi355x_tsan (ThreadSanitizer)")
    ap.add_argument("--checked", action="store_true",
                    help="also build the device-side debug build (_brp_checked, bin/einsteinbinary_mi355x_checked)")
    a = ap.parse_args(argv)
    out = build_with_checked(force=a.force, jobs=a.jobs) if a.checked else build(force=a.force, jobs=a.jobs)
    if a.asan:
        out["asan_app"] = str(build_asan(force=a.force, jobs=a.jobs))
    if a.tsan:
        out["tsan_app"] = str(build_tsan(force=a.force, jobs=a.jobs))
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
