"""CPU checks of the GPU formulation (tests/model_setops.py) against the oracle.

The kernels of bg_setops.hip compute set operations as running-max components, merge-path
pieces and replays; model_setops.py states the same construction in Python. These tests
compare it with oracle/bedops_oracle.c (the restatement of the reference's streaming
control flow, pinned by TestPlan.xml) on random inputs, so a formulation error shows up
here without a GPU.
"""
import os
import random
import subprocess
import tempfile

import pytest

import model_setops as M
import randbed


def _keyed(texts):
    rows = [[(ln.split("\t")[0], int(ln.split("\t")[1]), int(ln.split("\t")[2]))
             for ln in t.splitlines() if ln] for t in texts]
    names = sorted({c for f in rows for (c, _, _) in f}, key=lambda s: s.encode())
    rank = {n: i for i, n in enumerate(names)}
    keyed = [[((rank[c] << M.SHIFT) | s, (rank[c] << M.SHIFT) | e) for c, s, e in f] for f in rows]
    return keyed, names


def _render(pieces, names):
    mask = (1 << M.SHIFT) - 1
    return "".join(f"{names[s >> M.SHIFT]}\t{s & mask}\t{e & mask}\n" for s, e in pieces)


def _oracle(oracle_bin, args, texts, td):
    paths = []
    for i, t in enumerate(texts):
        p = os.path.join(td, f"in{i}.bed")
        with open(p, "w") as f:
            f.write(t)
        paths.append(p)
    return subprocess.run([oracle_bin["bedops"], *args, *paths], stdout=subprocess.PIPE,
                          check=True).stdout.decode()


@pytest.mark.parametrize("seed", range(4))
def test_model_intersect_zero_length_vs_oracle(oracle_bin, seed):
    """the zero-length replay of k_zi_replay, stated in Python, equals next_intersect"""
    rng = random.Random(seed)
    zero_prints = 0
    with tempfile.TemporaryDirectory() as td:
        for trial in range(150):
            nf = rng.choice([2, 2, 3, 4])
            texts = [randbed.text(randbed.rows(rng, rng.choice([0, 1, 3, 10, 40, 200]),
                                               span=rng.choice([30, 100, 400]),
                                               maxlen=rng.choice([3, 10, 40]),
                                               zero_frac=rng.choice([0.05, 0.2, 0.5])))
                     for _ in range(nf)]
            want = _oracle(oracle_bin, ["-i"], texts, td)
            keyed, names = _keyed(texts)
            got = _render(M.intersect_zero_len(keyed), names) if names else ""
            assert got == want, (seed, trial, texts)
            zero_prints += sum(1 for ln in want.splitlines() if ln.split("\t")[1] == ln.split("\t")[2])
    assert zero_prints > 0


@pytest.mark.parametrize("mode", ["-m", "-i", "-d"])
def test_model_setops_vs_oracle(oracle_bin, mode):
    """components / intersect2 / difference2 on inputs without zero-length rows"""
    rng = random.Random(hash(mode) & 0xffff)
    with tempfile.TemporaryDirectory() as td:
        for trial in range(80):
            nf = 1 if mode == "-m" else rng.choice([2, 3])
            texts = [randbed.text(randbed.rows(rng, rng.choice([0, 2, 30, 300]),
                                               span=rng.choice([50, 500]), maxlen=rng.choice([5, 60])))
                     for _ in range(nf)]
            want = _oracle(oracle_bin, [mode], texts, td)
            keyed, names = _keyed(texts)
            if not names:
                got = ""
            elif mode == "-m":
                got = _render(M.union_components(keyed), names)
            elif mode == "-i":
                acc = M.components(keyed[0])
                for f in keyed[1:]:
                    acc = M.intersect2(acc, M.components(f))
                got = _render(acc, names)
            else:
                got = _render(M.difference2(M.components(keyed[0]), M.union_components(keyed[1:])),
                              names)
            assert got == want, (mode, trial)


@pytest.mark.parametrize("ovr", [1, 3])
def test_model_bedmap_zero_length_window_vs_oracle(oracle_bin, ovr):
    """bedmap --count with zero-length rows: the window membership of k_mz_member"""
    rng = random.Random(ovr)
    with tempfile.TemporaryDirectory() as td:
        for trial in range(300):
            rs = randbed.rows(rng, rng.choice([1, 5, 30, 120]), span=rng.choice([40, 200]),
                              maxlen=rng.choice([5, 30]), zero_frac=rng.choice([0, 0.1, 0.4]),
                              chroms=["chr1", "chr2"])
            ms = randbed.rows(rng, rng.choice([1, 5, 30, 200]), span=rng.choice([40, 200]),
                              maxlen=rng.choice([5, 30, 100]), zero_frac=rng.choice([0, 0.1, 0.4]),
                              chroms=["chr1", "chr2"])
            paths = []
            for nm, rows in (("r", rs), ("m", ms)):
                paths.append(os.path.join(td, nm + ".bed"))
                with open(paths[-1], "w") as f:
                    f.write(randbed.text(rows))
            want = subprocess.run([oracle_bin["bedmap"], "--bp-ovr", str(ovr), "--count", *paths],
                                  stdout=subprocess.PIPE, check=True).stdout.decode().split()
            (kr, km), _ = _keyed([randbed.text(rs), randbed.text(ms)])
            zin, zout = M.bedmap_zero_len_window(kr, km)
            got = [str(sum(1 for j, (a, b) in enumerate(km)
                           if zin[j] is not None and zin[j] <= i < zout[j]
                           and min(e, b) - max(s, a) >= ovr and min(e, b) > max(s, a)))
                   for i, (s, e) in enumerate(kr)]
            assert got == want, (ovr, trial)
