#!/bin/bash
# round 5: where the tail's criterion-minima phase goes (measurement build: SKY_TINY_DBG 1 = no atomics, 2 = loads only)
O=gpurun_out/r05d
export SKYLINE_HIP_LIB=flink-skyline-qos_amd/build_measure/libskyline_hip.so SKY_TINY_CLK=1
for d in 0 1 2; do
  echo "== dbg $d"; SKY_TINY_DBG=$d timeout -k 10 120 python tools/tiny_debug.py mr-dim 0 2 1000000 8 2>&1 | grep tiny-clk || exit 1
done > ${O}_clk.txt 2>&1
