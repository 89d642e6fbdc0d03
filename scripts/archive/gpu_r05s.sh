#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
for m in plain numpy pytest conftest npz; do timeout -k 10 120 python3 scripts/dbg/drop_create_probe.py $m 2>&1 | grep create; done
