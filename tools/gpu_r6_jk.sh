#!/bin/bash
# round 6: lookahead from the compiler (GPU tests + drop-in), then the OFFSETS pipeline A/B
set -o pipefail
cd "$(dirname "$0")/.."
./tools/gpu_r6_j.sh && ./tools/gpu_r6_k.sh
