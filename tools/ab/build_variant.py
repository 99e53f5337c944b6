"""Build a libivc variant with extra compiler flags into ab/<name>.so (same sources and flags
as ivclab_amd/build.py):  python tools/ab/build_variant.py NAME [-DFOO=1 ...]
IVC_CSRC=<dir> compiles the sources from another directory (e.g. a copy holding an older
version of one file)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from ivclab_amd import build as B  # noqa: E402

name, extra = sys.argv[1], sys.argv[2:]
objdir = os.path.join("/tmp", "ivc_ab_" + name)
os.makedirs(objdir, exist_ok=True)
os.makedirs(os.path.join(ROOT, "ab"), exist_ok=True)
flags = [f for f in B.FLAGS if f != "-shared"] + extra
objs = [os.path.join(objdir, os.path.splitext(f)[0] + ".o") for f in B.SOURCES]
csrc = os.environ.get("IVC_CSRC", B.CSRC)
if csrc != B.CSRC:
    flags += ["-I" + B.CSRC]
jobs = [[B.hipcc()] + flags + B.FILE_FLAGS.get(f, []) + ["-c", "-o", o, os.path.join(csrc, f)]
        for f, o in zip(B.SOURCES, objs)]
with ThreadPoolExecutor(len(jobs)) as ex:
    list(ex.map(lambda c: B._run(c, False), jobs))
B._run([B.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
        os.path.join(ROOT, "ab", name + ".so")] + objs, False)
print(os.path.join("ab", name + ".so"))
