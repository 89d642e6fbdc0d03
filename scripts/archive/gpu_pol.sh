#!/bin/bash
# Mailbox record cache policy A/B at one basis length per library (ARN_NV_ONLY builds):
# sc1 (device scope) vs sc0 records, packed-halo baseline (NKHIP_ARN_MBOX=0).
set -o pipefail
for nv in 4 12 24; do
  bash scripts/arn_ab.sh $nv n${nv}p16:NKHIP_ARN_MBOX=0 n${nv}p16 n${nv}p1 || exit $?
done
