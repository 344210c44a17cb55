#!/bin/bash
# r06 h: lane-varying k_step2 on the stress pool vs the culling geometry (leaf size cull_chunk G,
# leaves per super cull_super SG); then the seed-1 pool at the same geometries (slot-uniform path)
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 400 python tools/r06/stress_probe.py 65536 lane_tracks=1 lane_tracks=1,cull_chunk=4 \
  lane_tracks=1,cull_chunk=4,cull_super=16 lane_tracks=1,cull_chunk=16,cull_super=4 lane_tracks=1,cull_super=4 \
  lane_tracks=1,cull_super=16 >> $O/probe.jsonl 2>> $O/probe.err
