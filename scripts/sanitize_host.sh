#!/bin/bash
# Host-side sanitizer runs (no GPU): the C oracle under UBSan across every
# golden-fixture test, and the engine's host selftest (LPM flattener, the
# self-traffic cut rule, prefix-mask known answers) under ASan + UBSan.
# Outputs go to /tmp only.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p /tmp/cfc_san
gcc -O1 -g -std=c11 -fPIC -shared -fopenmp -fsanitize=undefined -fno-sanitize-recover=undefined \
    -o /tmp/cfc_san/liboracle.so oracle/cfc_oracle.c
python - <<'PY'
import sys
sys.path[:0] = ["oracle", "tests", "."]
import oracle as O
O.LIB = "/tmp/cfc_san/liboracle.so"   # (the oracle loads its library lazily)
import pytest
sys.exit(pytest.main(["-x", "-q", "-p", "no:cacheprovider", "tests/test_oracle_golden.py"]))
PY
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-gpu-sanitize \
    -o /tmp/cfc_san/selftest cilium_amd/csrc/selftest.cpp cilium_amd/csrc/flatten.cpp \
    cilium_amd/csrc/maps.cpp
/tmp/cfc_san/selftest
