#!/bin/bash
# Copy the judged summaries of a GPU round out of gpurun_out/ (scratch) into profiles/ (tracked).
# usage: bash tools/collect_profiles.sh <round tag, e.g. r03_v4> [scan A/B tag, e.g. r03_scan1]
set -e
TAG=$1
SCAN=$2
src=gpurun_out/$TAG
if [ -d "$src" ]; then
  [ -s "$src/bench.json" ] && tail -1 "$src/bench.json" > "profiles/${TAG}_bench.json"
  [ -f "$src/prof/run_kernel_stats.csv" ] && cp "$src/prof/run_kernel_stats.csv" "profiles/${TAG}_kernel_stats.csv"
  [ -f "$src/replay_window.json" ] && cp "$src/replay_window.json" "profiles/${TAG}_replay_window.json"
  [ -f "$src/pmc_gemm.json" ] && cp "$src/pmc_gemm.json" "profiles/${TAG}_pmc_gemm.json"
  [ -f "$src/loop_events.txt" ] && grep -v amdgpu.ids "$src/loop_events.txt" > "profiles/${TAG}_loop_events.txt"
  [ -f "$src/predict_events.txt" ] && grep -v amdgpu.ids "$src/predict_events.txt" > "profiles/${TAG}_predict_events.txt"
fi
if [ -n "$SCAN" ] && [ -d "gpurun_out/$SCAN" ]; then
  s=gpurun_out/$SCAN
  [ -f "$s/c5.txt" ] && cp "$s/c5.txt" "profiles/${SCAN}_c5.txt"
  [ -f "$s/prof/run_kernel_stats.csv" ] && cp "$s/prof/run_kernel_stats.csv" "profiles/${SCAN}_w1_kernel_stats.csv"
  [ -f "$s/prof8/run_kernel_stats.csv" ] && cp "$s/prof8/run_kernel_stats.csv" "profiles/${SCAN}_w8_kernel_stats.csv"
fi
ls -la profiles | tail -12
