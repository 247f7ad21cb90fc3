import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from bedops_amd.engine import Engine, BedgpuError
eng = Engine()
for bad in (b"chr1\t50\t60\nchr1\t5\t10\n", b"chr2\t1\t2\nchr1\t1\t2\n",
            b"chr1\t1\t2\nchr2\t1\t2\nchr1\t3\t4\n", b"chr1\t50\t60\nchr1\t5\t10\nchr1\t70\t80\n"):
    try:
        out = eng.bedops("-m", [bad])
        print(os.environ.get("BEDGPU_SET_NT"), os.environ.get("BEDGPU_ROW_PARSE"), repr(bad), "NO ERROR", out)
    except BedgpuError as e:
        print(os.environ.get("BEDGPU_SET_NT"), os.environ.get("BEDGPU_ROW_PARSE"), repr(bad), "error", e.code, e)
