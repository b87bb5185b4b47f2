"""Run a script or pytest against a probe build of the library:
    python scripts/diag/with_lib.py <variant> bench.py [args...]
    python scripts/diag/with_lib.py <variant> -m pytest [args...]
(tools/probes/var/<variant>/libvideomamba_hip.so, scripts/diag/build_variant.py)."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import videomamba_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", sys.argv[1], "libvideomamba_hip.so")
if sys.argv[2] == "-m":
    sys.argv = [sys.argv[3]] + sys.argv[4:]
    runpy.run_module(sys.argv[0], run_name="__main__", alter_sys=True)
else:
    sys.argv = sys.argv[2:]
    runpy.run_path(sys.argv[0], run_name="__main__")
