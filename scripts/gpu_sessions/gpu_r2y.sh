#!/usr/bin/env bash
# Round-2 y: scripts/gpu_r2x.sh (masked-nibble FP4 gram) then scripts/gpu_r2w.sh (encode owner table).
d="$(dirname "$0")"
bash "$d/gpu_r2x.sh" && bash "$d/gpu_r2w.sh"
