"""reproduce test_bedmap_sharded_equals_single_device[int-echo...] outside pytest: the first
failing BEDGPU_DEVICES run's stderr (with AMD_LOG_LEVEL from the environment) to a file"""
import os, random, subprocess, sys, tempfile, zlib
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import randbed
from test_gpu_shard import CHROMS
case = ["--echo", "--echo-map-id", "--bases", "--median"]
rng = random.Random(zlib.crc32(repr((case, False)).encode()))
exe = os.path.join(os.path.dirname(__file__), "..", "bedops_amd", "bin", "bedmap")
with tempfile.TemporaryDirectory() as td:
    for trial in range(3):
        ref = randbed.rows(rng, rng.choice([1, 300, 2000]), chroms=rng.sample(CHROMS, rng.choice([1, 4, 9])), span=4000, maxlen=rng.choice([10, 120]))
        mp = randbed.rows(rng, rng.choice([1, 500, 3000]), chroms=rng.sample(CHROMS, rng.choice([1, 4, 9])), span=4000, maxlen=rng.choice([10, 120]))
        pr = randbed.write(os.path.join(td, f"r{trial}.bed"), randbed.text(ref, rest="cols", rng=rng))
        pm = randbed.write(os.path.join(td, f"m{trial}.bed"), randbed.text(mp, rest="bed5", rng=rng))
        for files in ([pr, pm], [pm]):
            for devs in (None, "0,0"):
                env = dict(os.environ)
                env.pop("BEDGPU_DEVICES", None)
                if devs:
                    env["BEDGPU_DEVICES"] = devs
                r = subprocess.run([exe, *case, *files], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=120)
                print(trial, len(files), devs, r.returncode, len(r.stdout), [len(open(f).read()) for f in files], flush=True)
                if r.returncode:
                    open("gpurun_out/isol/stderr.txt", "wb").write(r.stderr)
                    sys.exit(1)
