#!/bin/bash
# round 6: GPU suite + smoke on the current tree, HBM traffic passes (C4 new layout, U1-U3, W6), default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
PMC_CFGS="c4 u2 u3 w6 u1" bash scripts/gpu_ci.sh tests smoke pmc fullbench || exit 1
python3 scripts/pmc_to_json.py gpurun_out c4 u2 u3 w6 u1 --round r06
mkdir -p gpurun_out/r6 && cp profiles/pmc_c4.json profiles/pmc_u2.json profiles/pmc_u3.json profiles/pmc_w6.json profiles/pmc_u1.json gpurun_out/r6/
