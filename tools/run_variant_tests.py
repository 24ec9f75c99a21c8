"""Diagnostic: run GPU tests against an experiment-variant library
(build.py --out diag_exp/lib<X>.so -D...) instead of the in-tree product.
    python tools/run_variant_tests.py LIB.so [pytest args...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_forecasting_amd import _lib  # noqa: E402

_lib.load(sys.argv[1])
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[2:]))
