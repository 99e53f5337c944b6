"""Multi-core CPU baseline workers (TEST / MEASUREMENT INFRASTRUCTURE ONLY: used by
bench.py's cpu_baseline leg).  The reference is single-threaded; SURVEY.md §8d also asks for
the same NumPy path frame-sharded over the host's cores with multiprocessing — these are the
worker functions (module-level, so a spawn-context pool can import them without torch)."""
import os

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")


def warm(_):
    from . import ivc_oracle  # noqa: F401  (imports scipy once per worker)
    return os.getpid()


def intra_frames(frames):
    """The reference's intra path (oracle) on a list of [H, W] uint8 frames."""
    from . import ivc_oracle as O
    for f in frames:
        O.intra_encode(f[..., None], 1.0)
    return len(frames)


def me_stripe(args):
    """The reference's literal ME loop on a [rows, W] stripe pair (float64)."""
    from . import ivc_oracle as O
    a, b, sr = args
    O.motion_vectors_loop(a, b, sr)
    return a.shape[0]
