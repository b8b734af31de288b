#!/usr/bin/env bash
# Build the host runtime (no HIP) with sanitizers and run the self-test.
#   scripts/sanitize_host.sh asan   → AddressSanitizer + UndefinedBehaviorSanitizer
#   scripts/sanitize_host.sh tsan   → ThreadSanitizer (threaded miner / rules / generator)
# Host code only: GPU sanitizers are not available on the MI355X pool.
set -euo pipefail
cd "$(dirname "$0")/.."
mode=${1:-asan}
case "$mode" in
  asan) flags="-fsanitize=address,undefined -fno-sanitize-recover=undefined" ;;
  tsan) flags="-fsanitize=thread" ;;
  *) echo "usage: $0 asan|tsan" >&2; exit 2 ;;
esac
out=build/sanitize-$mode
mkdir -p "$out"
src="csrc/host/csv_encode.cpp csrc/host/miner_cpu.cpp csrc/host/matcher_cpu.cpp csrc/host/rules_cpu.cpp csrc/host/synth.cpp csrc/tests/host_selftest.cpp"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer $flags -Icsrc/include $src -o "$out/host_selftest" -pthread
"$out/host_selftest"
