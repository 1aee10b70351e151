"""tools/data_sweep.py against an alternative libtvam build: python tools/variant_data_sweep.py LIB.so N"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = [os.path.join(os.path.dirname(__file__), "data_sweep.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
