#!/bin/bash
# Attribution of the wide fused kernel (nv 12) by timing-only variants (results not valid):
# no packed halo load, no per-row barrier, no LDS lag.
set -o pipefail
bash scripts/arn_ab.sh ${ATTR_NV:-12} ${ATTR_VARIANTS:-xbase xnohalo xnobar xnolag}
