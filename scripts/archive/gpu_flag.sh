#!/bin/bash
# Mailbox pair kernel: block barrier vs LDS progress flags between its two waves (nv 24).
set -o pipefail
bash scripts/arn_ab.sh 24 base24 flag24
