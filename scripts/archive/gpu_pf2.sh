#!/bin/bash
# Rows in flight of the pair layout with 2-wave mailbox blocks (tuning builds, NKHIP_ARN_PF).
set -o pipefail
bash scripts/arn_ab.sh 24 t24:NKHIP_ARN_PF=1 t24:NKHIP_ARN_PF=2 || exit $?
bash scripts/arn_ab.sh 20 t20:NKHIP_ARN_PF=1 t20:NKHIP_ARN_PF=2 || exit $?
