"""In-tree build of the fscl_amd native library, the `fscl` CLI and the oracle.

    python -m fscl_amd.build            # everything
    python -m fscl_amd.build --no-oracle

Outputs (git-ignored, shipped to the GPU box with the snapshot):
    fscl_amd/_build/libfscl_amd.so   host C (gcc) + gfx950 HIP kernels (hipcc)
    fscl_amd/_build/fscl             drop-in CLI
    oracle/_build/*                  CPU restatement (test infrastructure)
    oracle/_ref/*                    reference subset, only where /root/reference exists

Flags: -O2 -ffp-contract=off for host C (the reference's canonical arithmetic),
-O3 -ffp-contract=off for the device code (no FMA contraction: bit-exactness).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "fscl_amd"
CSRC = PKG / "csrc"
OUT = PKG / "_build"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("FSCL_AMD_ARCH", "gfx950")

HOST_SRC = ["util.c", "input.c", "spectrum.c", "tables.c", "perm.c", "scan.c", "ranks.c"]
CFLAGS = ["-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-fopenmp", "-Wall", "-Wno-unused-result",
          "-std=gnu11"]
# iterative-ilp machine scheduling: 0.9 % (C2) / 0.4 % (C4) less time per launch, measured A/B
HIPFLAGS = [f"--offload-arch={ARCH}", "-O3", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-std=c++17",
            "-Wno-unused-value", "-Wno-unused-result", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]


def _run(cmd: list[str], cwd: Path | None = None) -> None:
    print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True, cwd=cwd)


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_native(force: bool = False, trace: bool = False, variant: str | None = None,
                 defines: tuple[str, ...] = ()) -> Path:
    """trace=True: a separate build in fscl_amd/_build_trace with device printf tracing;
    variant/defines: an experiment build in fscl_amd/_build_<variant> with extra -D flags."""
    global OUT
    out_saved = OUT
    if trace:
        OUT = PKG / "_build_trace"
    elif variant:
        OUT = PKG / f"_build_{variant}"
    try:
        return _build_native(force, trace, defines)
    finally:
        OUT = out_saved


def _build_native(force: bool, trace: bool, defines: tuple[str, ...] = ()) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    # every header a source may include (csrc/host/*.h: fscl_host.h, rows_impl.h, ...; csrc/device/*.h) and this file (the flags)
    hdrs = list((ROOT / "include").glob("*.h")) + sorted((CSRC / "host").glob("*.h")) + sorted((CSRC / "device").glob("*.h")) + [Path(__file__)]
    objs = []
    for src in HOST_SRC:
        s = CSRC / "host" / src
        o = OUT / (s.stem + ".o")
        if force or _stale(o, [s, *hdrs]):
            _run(["gcc", *CFLAGS, *defines, "-c", s, "-o", o])
        objs.append(o)
    hip_src = CSRC / "device" / "fsclg.hip"
    hip_obj = OUT / "fsclg.o"
    if force or _stale(hip_obj, [hip_src, *hdrs]):
        _run([ROCM / "bin" / "hipcc", *HIPFLAGS, *(["-DFSCLG_TRACE"] if trace else []), *defines, "-c", hip_src, "-o", hip_obj])
    objs.append(hip_obj)
    lib = OUT / "libfscl_amd.so"
    if force or _stale(lib, objs):
        _run(["g++", "-shared", "-o", lib, *objs, f"-L{ROCM / 'lib'}", "-lamdhip64", "-lgomp", "-lm", "-lpthread",
              f"-Wl,-rpath,{ROCM / 'lib'}"])
    cli = OUT / "fscl"
    main_src = CSRC / "host" / "fscl_main.c"
    if force or _stale(cli, [main_src, lib, *hdrs]):
        _run(["gcc", *CFLAGS, "-o", cli, main_src, f"-L{OUT}", "-lfscl_amd", "-lm", "-Wl,-rpath,$ORIGIN"])
    return lib


def build_oracle() -> None:
    make = shutil.which("make")
    if not make:
        raise RuntimeError("make not found")
    _run([make, "-s", "-C", ROOT / "oracle", "all"])
    if Path("/root/reference").is_dir():
        _run([make, "-s", "-C", ROOT / "oracle", "ref"])


def main(argv: list[str]) -> int:
    force = "--force" in argv
    build_native(force=force)
    if "--trace" in argv:
        build_native(force=force, trace=True)
    if "--rehearsal" in argv:  # the scaling-rehearsal test build (tools/scale_sim.sh)
        build_native(force=force, variant="rehearsal", defines=("-DFSCL_AMD_REHEARSAL",))
    if "--logx" in argv:  # the computed mid-branch log distance (FSCLG_LOG_CALC): 2 in every
        # kernel, 1 in the split kernel only; and their rehearsal builds
        for v, lc in (("logx", "2"), ("logxs", "1")):
            build_native(force=force, variant=v, defines=(f"-DFSCLG_LOG_CALC={lc}",))
            build_native(force=force, variant=f"rehearsal_{v}", defines=("-DFSCL_AMD_REHEARSAL", f"-DFSCLG_LOG_CALC={lc}"))
    for a in argv:  # --variant=NAME:DEF[,DEF...]: an experiment build fscl_amd/_build_NAME with -DDEF each
        if a.startswith("--variant="):
            name, _, defs = a[len("--variant="):].partition(":")
            build_native(force=force, variant=name, defines=tuple(f"-D{d}" for d in defs.split(",") if d))
    if "--no-oracle" not in argv:
        build_oracle()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
