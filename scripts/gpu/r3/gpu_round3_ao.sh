#!/bin/bash
# Per-call public API on gfx950: where the CPU goes (cProfile), device vs host.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r3ao
timeout -k 10 240 python -u scripts/api_percall_prof.py --device cuda --n 10000 > gpurun_out/r3ao/cuda.txt 2>&1 &&
timeout -k 10 240 python -u scripts/api_percall_prof.py --device host --n 10000 > gpurun_out/r3ao/host.txt 2>&1
