#!/bin/bash
# Experiment: vector-pair layout with 2-wave (128-column) blocks + mailbox vs 4-wave blocks, nv 24
# (no edge arrays in either: the 2-wave build's edge-array geometry differs from the library's).
set -o pipefail
bash scripts/arn_ab.sh 24 w4b:ARN_EDGES=0 w2b:ARN_EDGES=0
