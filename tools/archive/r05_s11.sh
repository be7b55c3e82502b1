#!/bin/bash
# round 5 session 11: every -m gpu test (incl. the 8-RX MMSE cases), then the TX bin-mapping share
# (trivial-bins timing variant, output meaningless) against the base build
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
NO_PMC=1 tools/ab_lib_pmc.sh base txtb
