#!/bin/bash
# Experiment: wide layout with 2-wave (256-column) blocks, plain and with the mailbox, vs 4-wave.
set -o pipefail
for nv in 4 12; do
  bash scripts/arn_ab.sh $nv w4n$nv w2n$nv w2mn$nv || exit $?
done
bash scripts/arn_ab.sh 24 m2n24 m1n24 || exit $?
