#!/bin/bash
# closing measurement (tools/final_r06.sh) followed by the C4 PMC pass of the same build
set -e
bash tools/final_r06.sh
bash tools/profile_r03.sh r06_c4 --batch 16384
