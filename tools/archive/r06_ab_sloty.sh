#!/bin/bash
# rx_epoch with the epoch's Y rows in a small set of packet images (XS_EP_SLOTY, timing only)
set -e
bash tools/ab_lib.sh default sloty default sloty
