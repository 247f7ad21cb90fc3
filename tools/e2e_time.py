#!/usr/bin/env python3
"""Run a command with its stdout to a file and split its wall clock with the CLI's
BEDGPU_STATS marks: spawn -> "start" mark (process start, loader, argv), the marked
phases, "exit" mark -> the parent sees the process end (teardown).
usage: e2e_time.py <out-file> <cmd...>"""
import os
import subprocess
import sys
import time

env = dict(os.environ, BEDGPU_STATS="1")
with open(sys.argv[1], "wb") as fo:
    t0 = time.monotonic()
    p = subprocess.run(sys.argv[2:], stdout=fo, stderr=subprocess.PIPE, env=env)
    t1 = time.monotonic()
err = p.stderr.decode()
mono = {ln.split()[2]: float(ln.split()[3]) for ln in err.splitlines() if ln.startswith("bedgpu mono")}
sys.stderr.write(err)
if "start" in mono and "exit" in mono:
    sys.stderr.write(f"split: before-start {1e3 * (mono['start'] - t0):.1f} ms, marked "
                     f"{1e3 * (mono['exit'] - mono['start']):.1f} ms, after-exit {1e3 * (t1 - mono['exit']):.1f} ms, "
                     f"total {1e3 * (t1 - t0):.1f} ms\n")
sys.exit(p.returncode)
