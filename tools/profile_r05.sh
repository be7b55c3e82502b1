#!/bin/bash
# Round-5 PMC profiles (tools/profile_r03.sh per workload) of the closing build: the default C4 bench
# step (one 16384-slot chunk), the C4SM (MMSE) step (4096) and the C4 step with the fused PDC receiver.
# -> gpurun_out/prof_r05_<tag>/
set -e
bash tools/profile_r03.sh r05_c4 --batch 16384
bash tools/profile_r03.sh r05_c4sm --workload C4SM --batch 8192
DNRP_RX_FUSED=1 bash tools/profile_r03.sh r05_fused --batch 16384
