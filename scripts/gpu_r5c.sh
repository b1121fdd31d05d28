#!/bin/bash
# Round-5 GPU session 2: comm stream kind A/B and the BN-apply ceiling experiment.
set -o pipefail
bash scripts/diag/ab_comm_stream.sh && bash scripts/diag/ab_skip_bn.sh
