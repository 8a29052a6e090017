#!/bin/bash
# Round 6's final evidence in two gpurun calls (each well under 20 minutes):
#   tools/r6_final.sh prof   rocprofv3 stats + FETCH / WRITE / SQ passes for C3, C2, C5 and the
#                            driver command's kernel trace (tools/round_evidence.sh's prof part)
#   tools/r6_final.sh bench  GPU suite, the driver's command, 400-step C3, C5, C2, entropy index,
#                            two ranks on one GPU (its bench part)
# The prof part writes gpurun_out/sq_*.json / traffic_*.json, which bench.py's
# roofline reads from profiles/: run prof first and copy them in.
TAG=${TAG:-r6x}
PART=${1:-bench}
bash tools/round_evidence.sh $TAG $PART
