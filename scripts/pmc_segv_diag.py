"""Run bench.py in this process with tools/segv_maps.so loaded (diagnostic for the r4i crash under
rocprofv3 --pmc: on SIGSEGV the faulting address, dladdr-named frames and /proc/self/maps go to
stderr before the profiler's own handler runs). Usage: python3 scripts/pmc_segv_diag.py <bench args>"""
import ctypes
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ctypes.CDLL(os.path.join(ROOT, "tools", "segv_maps.so"))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
