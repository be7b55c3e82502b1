#!/bin/bash
# Round-6 PMC profiles (tools/profile_r03.sh per workload) of the closing build: the default C4 bench
# step (one 16384-slot chunk, epoch receiver), the C4 step through the Y path (DNRP_RX_EPOCH=0) and the
# C4SM (MMSE) step (8192). -> gpurun_out/prof_r06_<tag>/
set -e
bash tools/profile_r03.sh r06_c4 --batch 16384
DNRP_RX_EPOCH=0 bash tools/profile_r03.sh r06_ypath --batch 16384
bash tools/profile_r03.sh r06_c4sm --workload C4SM --batch 8192
