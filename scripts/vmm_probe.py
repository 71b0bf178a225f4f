#!/usr/bin/env python3
"""Run tools/vmm_probe's exporter and importer as two child processes on the
one GPU (this parent never touches the GPU) and print both outputs.

    python scripts/vmm_probe.py [MiB = 64]
"""
import os
import subprocess
import sys
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
exe = os.path.join(ROOT, "tools", "vmm_probe")
mib = sys.argv[1] if len(sys.argv) > 1 else "64"
name = f"xucg_vmm_probe_{os.getpid()}_{uuid.uuid4().hex[:6]}"
ex = subprocess.Popen([exe, "export", name, mib], stdout=subprocess.PIPE,
                      stderr=subprocess.STDOUT, text=True)
im = subprocess.Popen([exe, "import", name, mib], stdout=subprocess.PIPE,
                      stderr=subprocess.STDOUT, text=True)
rc = 0
for tag, p in (("import", im), ("export", ex)):
    try:
        out, _ = p.communicate(timeout=120)
    except subprocess.TimeoutExpired:
        p.kill()
        out, _ = p.communicate()
        out += "\n<killed: timeout>"
    print(f"=== {tag} (exit {p.returncode})\n{out}", flush=True)
    rc = rc or p.returncode
sys.exit(rc)
