#!/usr/bin/env python3
"""Run GPU steps one after another on the box, each under its own time limit.

Stops at the first step that ends with a crash-like status (fault, abort, segfault, time
limit): nothing else touches the GPU after that. Ordinary failures (exit 1, e.g. a failing
assertion) do not stop later steps. Output of step i goes to gpurun_out/<name>.log.
Usage: gpu_steps.py name1 seconds1 'cmd1' [name2 seconds2 'cmd2' ...]
"""
import os
import subprocess
import sys
import time

args = sys.argv[1:]
os.makedirs("gpurun_out", exist_ok=True)
for i in range(0, len(args), 3):
    name, secs, cmd = args[i], int(args[i + 1]), args[i + 2]
    t0 = time.time()
    with open(f"gpurun_out/{name}.log", "w") as f:
        r = subprocess.run(["timeout", "-k", "10", str(secs), "bash", "-c", cmd], stdout=f, stderr=subprocess.STDOUT)
    rc = r.returncode
    print(f"[{name}] rc={rc} {time.time() - t0:.1f}s", flush=True)
    with open(f"gpurun_out/{name}.log") as f:
        tail = f.read()[-1500:]
    print(tail, flush=True)
    if rc not in (0, 1, 2, 5):
        print(f"[{name}] crash-like status {rc}: stopping", flush=True)
        sys.exit(rc)
