"""The sparse path's own kernel sources run on the CPU wave emulator (csrc/emu: a host thread per
lane, block barriers, the launch's dynamic LDS) under AddressSanitizer and UBSan:

* level-2 pair rows (csrc/kernels/pairrows.hip: frequent-rank filters with per-wave pooled
  reservations, pair-list passes A/B direct and staged, LDS row counts) — the gram must equal a
  host loop's co-occurrence counts;
* the horizontal levels (csrc/kernels/hlevels.hip: filtered CSR, hit lists, the candidate hash
  table's CAS insert, flat wave probes with per-wave slot blocks, trie compaction) — every
  frequent itemset of size >= 2 and its support must equal a host tid-list miner's."""
import json
import os
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
BIN = ROOT / "build" / "emu" / "pairrows_emu"
HL_BIN = ROOT / "build" / "emu" / "hlevels_emu"


def _build(BIN=BIN, kernel="pairrows", main_src="pairrows_emu_main.cpp"):
    srcs = [ROOT / f"csrc/kernels/{kernel}.hip"]
    main = ROOT / "csrc/tests" / main_src
    deps = srcs + [main] + list((ROOT / "csrc/emu").rglob("*")) + \
        list((ROOT / "csrc/include").rglob("*.hpp")) + \
        [ROOT / "csrc/kernels/kernels.hpp", ROOT / "csrc/kernels/devbuf.hpp"]
    newest = max(p.stat().st_mtime for p in deps if p.is_file())
    if BIN.exists() and BIN.stat().st_mtime >= newest:
        return
    BIN.parent.mkdir(parents=True, exist_ok=True)
    import fcntl
    with open(BIN.parent / f".build_{kernel}.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if BIN.exists() and BIN.stat().st_mtime >= newest:
            return
        tmp = BIN.with_name(f"{BIN.name}.{os.getpid()}.tmp")
        cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
               "-fno-omit-frame-pointer", f"-I{ROOT / 'csrc/emu'}", f"-I{ROOT / 'csrc/include'}",
               "-x", "c++"] + [str(s) for s in srcs] + ["-x", "none", str(main), "-lpthread",
                                                        "-o", str(tmp)]
        subprocess.run(cmd, check=True, capture_output=True, timeout=600)
        os.replace(tmp, BIN)


@pytest.fixture(scope="module")
def pr_bin():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    _build()
    return BIN


@pytest.fixture(scope="module")
def hl_bin():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    _build(HL_BIN, "hlevels", "hlevels_emu_main.cpp")
    return HL_BIN


@pytest.mark.parametrize("args", [
    # n_tx n_items max_len seed hooks fmask world
    "600 70 12 1 - 1 1",                      # LDS-mask filter (16 waves), staged pass B
    "600 70 12 2 filter_lds=0 1 1",           # mask in L2 (8-wave instance)
    "600 70 12 3 pl_staged=0 0 1",            # per-lane filter, direct passes A and B
    "500 60 30 4 pl_staged_a=1,pl_groups=3 1 1",  # staged pass A, long rows, 3 groups
    "600 70 10 5 - 1 2",                      # item-sharded: owned rows a % 2 == 0
])
def test_pairrows_on_emulator(pr_bin, args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1")
    p = subprocess.run([str(pr_bin)] + args.split(), capture_output=True, text=True,
                       timeout=900, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["bad"] == 0 and out["pairs"] > 0 and out["F"] > 20, out


@pytest.mark.parametrize("args", [
    # n_tx n_items max_len seed min_count hooks
    "500 40 14 2 8 -",            # sizes up to 9
    "600 50 16 3 6 hl_cap=64",    # tiny initial capacities: every re-count / regrow path
])
def test_hlevels_on_emulator(hl_bin, args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1")
    p = subprocess.run([str(hl_bin)] + args.split(), capture_output=True, text=True,
                       timeout=900, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["bad"] == 0 and out["itemsets"] > 1000 and out["max_depth"] >= 5, out
