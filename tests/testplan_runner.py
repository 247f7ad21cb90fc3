"""Runner for the reference's bedops KATs (tests/golden/testplan.json).

Restates Regression.java's semantics (applications/bed/bedops/test/Regression.java:
27-90 runner, :150-177 Perform): tests run in `order`; every test's INPUT files are
written first; the command is `<bedops> --ec <CALL> <input files...>`; a non-zero
exit or ANY stderr output fails the test; stdout lines are trim()'ed, empty lines
dropped, the result is written to the test's OUTPUT file (later tests read it) and
string-compared with the ANSWER.
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "testplan.json")

# mode letters of each KAT's operation (first CALL token)
_MODE = {"-m": "m", "--merge": "m", "-i": "i", "--intersect": "i", "-d": "d",
         "--difference": "d", "-e": "e", "--element-of": "e", "-n": "n",
         "--not-element-of": "n", "-c": "c", "--complement": "c", "-s": "s",
         "--symmdiff": "s", "-u": "u", "--everything": "u", "-p": "p",
         "--partition": "p", "-w": "w", "--chop": "w"}


def load_tests():
    with open(FIXTURE) as f:
        return json.load(f)["tests"]


def test_mode(t):
    for tok in t["call"]:
        if tok in _MODE:
            return _MODE[tok]
    return None


def run_testplan(bedops_cmd, workdir, modes=None, env=None):
    """Run every KAT (those whose mode is in `modes`, if given) with `bedops_cmd`
    (a list of argv words). Returns a list of (order, call, passed, detail)."""
    tests = load_tests()
    os.makedirs(workdir, exist_ok=True)
    results = []
    for t in tests:
        for inp in t["inputs"]:
            with open(os.path.join(workdir, inp["name"]), "w") as f:
                f.write(inp["data"])
    for t in tests:
        m = test_mode(t)
        if modes is not None and m not in modes:
            # not exercised here: later tests may read its OUTPUT file, which the
            # reference (63/63 passing) leaves equal to its ANSWER
            with open(os.path.join(workdir, t["output"]), "w") as f:
                f.write(t["answer"])
            continue
        argv = list(bedops_cmd) + ["--ec"] + t["call"] + [i["name"] for i in t["inputs"]]
        p = subprocess.run(argv, cwd=workdir, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           env=env, timeout=120)
        out = "".join(ln.strip() + "\n" for ln in p.stdout.decode().split("\n")
                      if len(ln) > 0)
        with open(os.path.join(workdir, t["output"]), "w") as f:
            f.write(out)
        err = p.stderr.decode()
        ok = p.returncode == 0 and err == "" and out == t["answer"]
        detail = "" if ok else f"rc={p.returncode} err={err[:200]!r} got={out[:300]!r} want={t['answer'][:300]!r}"
        results.append((t["order"], " ".join(t["call"]), ok, detail))
    return results
