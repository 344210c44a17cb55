#!/bin/bash
# Same-session sweep of the raycast culling granularity (leaf chunk G, super-chunk SG) on the bench workload
set -u
AB_SETS="${SETS:-c8s8|| --cull-chunk 8 --cull-super 8;c12s6|| --cull-chunk 12 --cull-super 6;c16s4|| --cull-chunk 16 --cull-super 4;c16s8|| --cull-chunk 16 --cull-super 8;c6s8|| --cull-chunk 6 --cull-super 8;c8s6|| --cull-chunk 8 --cull-super 6;c8s12|| --cull-chunk 8 --cull-super 12;c10s8|| --cull-chunk 10 --cull-super 8}" bash tools/ab_args.sh
