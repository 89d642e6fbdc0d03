#!/bin/bash
# Lag-row prefetch of the pair layout (ARN_LAGPRE_MAX builds): off vs on at nv 20 and 24.
set -o pipefail
bash scripts/arn_ab.sh 20 l0n20 l22n20 || exit $?
bash scripts/arn_ab.sh 24 l0n24 l26n24 || exit $?
