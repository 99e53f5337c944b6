"""Turn a FETCH_SIZE / WRITE_SIZE PMC summary (tools/pmc_reduce.py output) into the per-launch
HBM traffic record bench.py reports as roofline.traffic (profiles/pmc_intra_latest.json).

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): the
counters are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane)
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def csrc_sha256():
    """Same key as bench.csrc_sha256: the HIP sources libivc is built from."""
    d = os.path.join(ROOT, "ivclab_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".h")):
            with open(os.path.join(d, f), "rb") as fh:
                h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()


def main(summary, frames, H, W, out,
         match="fused_encode_kernel<unsigned char, double, double, 1, true, false, 0,"):
    d = json.load(open(summary))
    name = next(k for k in d if match in k)
    rec = d[name]
    fetch = rec["FETCH_SIZE"]["mean"] * 1024
    write = rec["WRITE_SIZE"]["mean"] * 1024
    frames, H, W = int(frames), int(H), int(W)
    res = {"kernel": name, "frames": frames, "H": H, "W": W,
           "fetch_bytes_raw": fetch, "fetch_bytes_corrected": 2 * fetch, "write_bytes": write,
           "hbm_bytes_per_launch": 2 * fetch + write,
           "algorithmic_bytes_per_launch": 13 * frames * H * W,
           "dispatches": rec["FETCH_SIZE"]["n"],
           "note": "FETCH_SIZE x2 (gfx950 wide-read correction), WRITE_SIZE as is; KiB -> bytes",
           "csrc_sha256": csrc_sha256(),
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of the bench kernel "
                     "(committed record, keyed by the csrc hash)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
