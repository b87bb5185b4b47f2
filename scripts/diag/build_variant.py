"""Build a probe variant of libvideomamba_hip.so: copy csrc/ to build/var/<name>/, apply the
variant's text replacements, build to tools/probes/var/<name>/libvideomamba_hip.so.  Product
sources stay untouched; scripts/diag/variant_scan.py loads a variant by path.
    python scripts/diag/build_variant.py bc_fixed
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name -> [(file, old, new)]
VARIANTS = {
    # timing probe: every step reads the segment's first B/C row (L1/K$-resident), so the
    # chunk kernel's time without the per-step scalar-load latency shows (results wrong)
    "bc_fixed": [("vm_scan_seq.hip",
                  "      bc_load(min(t + 1, tlast), bcw[(j + 1) & 1]);",
                  "      bc_load(t_beg, bcw[(j + 1) & 1]);")],
}


def build(name):
    src = os.path.join(ROOT, "videomamba_amd", "csrc")
    work = os.path.join(ROOT, "build", "var", name, "src", "csrc")  # ../../include resolves
    shutil.rmtree(work, ignore_errors=True)
    shutil.copytree(src, work)
    inc = os.path.join(ROOT, "build", "var", name, "include")
    shutil.rmtree(inc, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "include"), inc)
    for fname, old, new in VARIANTS[name]:
        p = os.path.join(work, fname)
        s = open(p).read()
        assert s.count(old) >= 1, (name, fname, old)
        open(p, "w").write(s.replace(old, new))
    out = os.path.join(ROOT, "tools", "probes", "var", name)
    os.makedirs(out, exist_ok=True)
    subprocess.check_call(["make", "-C", work, "-j8", f"OUT={out}/libvideomamba_hip.so",
                           f"BUILD={os.path.join(ROOT, 'build', 'var', name, 'obj')}"])


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
