"""bench.py against another build of the engine (A/B of two libraries on one box): GX_LIB names
the library that load_product() returns in this process."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import sidecar_amd.abi as abi  # noqa: E402

path = os.path.join(ROOT, os.environ["GX_LIB"])
abi.load_product = lambda: abi.load_library(path)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
