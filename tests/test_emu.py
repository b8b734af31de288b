"""The count-only deep GPU miner's own kernel source, run on the CPU wave emulator (csrc/emu).

csrc/kernels/deep.hip and csrc/host/deep_run.hip are compiled by g++ against the emulator's HIP
shim (one host thread per lane, cross-lane ops through barriers) with AddressSanitizer and
UBSan; the per-size counts and the content digest must equal the CPU count miner's.  Small step
budgets force spills (in-launch work stealing, or spill rounds); world > 1 splits the level-3 tasks over simulated ranks; longer
transaction lists exercise the tid projection across several width tiers.
"""
import os
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
BIN = ROOT / "build" / "emu" / "deep_emu"


def _build():
    srcs = [ROOT / "csrc/kernels/deep.hip", ROOT / "csrc/host/deep_run.hip"]
    host = [ROOT / f"csrc/host/{f}" for f in ("miner_cpu.cpp", "synth.cpp", "digest.cpp")]
    main = ROOT / "csrc/tests/deep_emu_main.cpp"
    host.append(ROOT / "csrc/tests/deep_order_emu.cpp")  # stand-in for the hipCUB task sort
    deps = srcs + host + [main] + list((ROOT / "csrc/emu").rglob("*")) + \
        list((ROOT / "csrc/include").rglob("*.hpp")) + [ROOT / "csrc/kernels/kernels.hpp",
                                                        ROOT / "csrc/host/deep_run.hpp"]
    newest = max(p.stat().st_mtime for p in deps if p.is_file())
    if BIN.exists() and BIN.stat().st_mtime >= newest:
        return
    BIN.parent.mkdir(parents=True, exist_ok=True)
    # parallel test workers (pytest -n): one builds under an exclusive lock, into a temp file
    # renamed over the binary, so no worker executes a half-written file
    import fcntl
    with open(BIN.parent / ".build.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if BIN.exists() and BIN.stat().st_mtime >= newest:
            return
        tmp = BIN.with_name(f"{BIN.name}.{os.getpid()}.tmp")
        cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
               "-fno-omit-frame-pointer", f"-I{ROOT / 'csrc/emu'}", f"-I{ROOT / 'csrc/include'}",
               "-x", "c++"] + [str(s) for s in srcs] + ["-x", "none"] + [str(h) for h in host] + \
              [str(main), "-lpthread", "-o", str(tmp)]
        subprocess.run(cmd, check=True, capture_output=True, timeout=600)
        os.replace(tmp, BIN)


@pytest.fixture(scope="module")
def emu_bin():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    _build()
    return BIN


@pytest.mark.parametrize("args", [
    # n_tx n_items mean_len genres affinity min_support [budget0 budget split_min stack_mb world
    #   max_len steal steal_idle presplit_cost emit]   (n_items < 0: a clique of -n_items items)
    "400 60 20 3 0.9 0.05",
    "400 60 20 3 0.9 0.05 1 1 2 4 1 0 1 0",          # steal: every check spills, per-member splits
    "300 50 25 2 0.95 0.08 1 1 4 1 3 0 1 0",         # 3 simulated ranks + eager in-launch spills
    "300 50 25 2 0.95 0.08 4 4 64 1 1 4",            # max_len
    "1500 60 16 3 0.9 0.06 2 2 4 4 1 0 1 0",         # 24-word root: projected tiers 3..12 below it
    "400 60 20 3 0.9 0.05 1 1 2 4 1 0 0",            # spill rounds (steal off): every task spills
    "300 50 25 2 0.95 0.08 1 2 4 1 3 0 0",           # spill rounds, 3 simulated ranks
    "64 -13 1 1 1 0.5 1 2 8 4 1 0 1 2",              # clique of 13 items, partner hand-offs
    "64 -12 1 1 1 0.5 1 1 8 4 3 0 1 1",              # clique, 3 ranks, requested hand-offs
    "400 60 20 3 0.9 0.05 1 4 2 4 2 0 1 1 2",        # 2 ranks, pre-split of every task >= 2
    "64 -12 1 1 1 0.5 1 4 4 4 2 0 1 1 1",            # clique, 2 ranks: pre-split, then stealing
    "400 60 20 3 0.9 0.05 1 1 2 4 1 0 1 1 16 1",     # emit: the node arena's own digest
    "300 50 25 2 0.95 0.08 1 2 4 1 3 0 1 1 2 1",     # emit, 3 ranks, pre-split + hand-offs
    "64 -12 1 1 1 0.5 1 4 4 4 1 0 0 0 0 1",          # emit through spill rounds (steal off)
])
def test_deep_kernel_on_emulator(emu_bin, args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([str(emu_bin)] + args.split(), capture_output=True, text=True,
                       timeout=900, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert '"ok": true' in r.stdout


@pytest.mark.parametrize("args", [
    "64 -13 1 1 1 0.5 1 2 8 4 1 0 1 2",              # clique of 13, partner hand-offs
    "64 -12 1 1 1 0.5 1 1 8 4 3 0 1 1",              # clique, 3 ranks, requested hand-offs
    "300 50 25 2 0.95 0.08 1 2 4 1 3 0 1 1 2 1",     # emit, 3 ranks, pre-split + hand-offs
])
def test_deep_split_handoffs_on_emulator(emu_bin, args):
    """Hand-offs that split classes (donate_bottom: the upper members go, the frame keeps a lead
    of first members) at every size from 2 first members, so the small emulator problems split
    and re-split frames that already carry a lead — counts and digests still exact."""
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0",
               KMLS_TEST_HOOKS="deep_split_firsts=2,deep_split_keep16=8")
    r = subprocess.run([str(emu_bin)] + args.split(), capture_output=True, text=True,
                       timeout=900, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert '"ok": true' in r.stdout
