#!/bin/bash
# Regenerates the reference-answered fixtures (build container only: needs
# /root/reference and the conda Python 3.9 that has PLY 3.11).
#   step 1: seeded synthetic KB texts + query lists (this repo's generators)
#   step 2: the reference itself loads and answers them (make_golden.py)
set -euo pipefail
cd "$(dirname "$0")/../.."
export DAS_GOLDEN_SCRATCH=${DAS_GOLDEN_SCRATCH:-/tmp/das_golden}
export PYTHONDONTWRITEBYTECODE=1
python tests/golden/make_synthetic.py
/opt/conda/bin/python3.9 tests/golden/make_golden.py "${@:-synthetic}"
