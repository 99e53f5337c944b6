"""Turn a FETCH_SIZE / WRITE_SIZE PMC summary (tools/pmc_reduce.py output) into the per-launch
HBM traffic record bench.py reports as roofline.traffic (profiles/pmc_intra_latest.json).

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): the
counters are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane)
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores."""
import json
import sys


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
           "note": "FETCH_SIZE x2 (gfx950 wide-read correction), WRITE_SIZE as is; KiB -> bytes"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
