#!/bin/bash
# Round-4 PMC profiles (tools/profile_r03.sh per workload): the default C4 bench step, the C4SM (MMSE)
# step and the C4 step with the fused PDC receiver (DNRP_RX_FUSED=1), each one chunk of the workload's
# default size (C4: 16384 slots, C4SM: 4096). -> gpurun_out/prof_r04_<tag>/
set -e
bash tools/profile_r03.sh r04_c4 --batch 16384
bash tools/profile_r03.sh r04_c4sm --workload C4SM
DNRP_RX_FUSED=1 bash tools/profile_r03.sh r04_fused --batch 16384
