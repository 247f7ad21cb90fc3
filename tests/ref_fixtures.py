"""Loader + runner for the reference-produced fixtures (tests/golden/ref_*.json.gz,
made by tests/golden/make_ref_fixtures.py from the genuine reference built by
oracle/build_ref.sh). Used by tests/test_ref_fixtures.py (oracle vs reference, CPU) and
tests/test_gpu_ref_fixtures.py (the GPU drop-in CLIs vs reference)."""
import gzip
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
SUITES = ["closest", "bedmap", "decimal", "sortbed", "ec", "faster", "f2", "r6"]


def load(suite):
    with gzip.open(os.path.join(HERE, "golden", f"ref_{suite}.json.gz"), "rb") as f:
        return json.loads(f.read().decode())


def run_case(binary, fx, case):
    """(stdout, stderr, rc) of `binary` on one case, stderr with temp paths masked"""
    texts = fx["groups"][case["group"]]
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for i, t in enumerate(texts):
            p = os.path.join(td, f"in{i}.bed")
            with open(p, "w") as f:
                f.write(t)
            paths.append(p)
        argv = [binary] + case["args"] + [paths[i] if i >= 0 else "-" for i in case["files"]]
        stdin = texts[case["stdin"]].encode() if case.get("stdin") is not None else None
        r = subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, input=stdin, timeout=120)
    err = r.stderr.decode(errors="replace")
    for i, p in enumerate(paths):
        err = err.replace(p, f"@{i}")
    return r.stdout.decode(errors="surrogateescape"), err, r.returncode


def compare(binary, fx, case, check_stderr=True):
    """None when `binary` reproduces the case, else a short description of the difference"""
    out, err, rc = run_case(binary, fx, case)
    if out != case["stdout"]:
        a, b = out.splitlines(), case["stdout"].splitlines()
        for i, (x, y) in enumerate(zip(a, b)):
            if x != y:
                return f"stdout line {i + 1}: got {x!r} want {y!r}"
        return f"stdout: got {len(a)} lines want {len(b)}"
    if (rc == 0) != (case["rc"] == 0):
        return f"rc {rc} want {case['rc']} (stderr {err!r})"
    if check_stderr and err != case["stderr"]:
        return f"stderr {err!r} want {case['stderr']!r}"
    return None
