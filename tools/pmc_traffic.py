"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc rocpd databases
(FETCH_SIZE pass, WRITE_SIZE pass), keyed by the short kernel names bench.py's
HIP-event scopes use.

    python tools/pmc_traffic.py <fetch-dir> <write-dir> [steps]

FETCH_SIZE and WRITE_SIZE are reported in KiB.  FETCH_SIZE counts 64 B per
memory request (profiles/fetch_calibration.json, tools/ubench/fetch_cal.hip):
a wide coalesced stream issues 128-B requests tallied at 64 B, so streaming
kernels' reads are 2 x FETCH_SIZE (MI355X_MICROARCH.md, HBM); an isolated
4-B load is one 64-B request counted exactly, so the random-probe and
random-gather kernels (RANDOM below) take FETCH_SIZE as is.  The raw figure is reported beside the
corrected one.  WRITE_SIZE is used as is.
TOPK=k (env) averages only each kernel's k largest launches (the timed
full-size launches of a run whose warm-up step is a small KB, e.g. the build).
"""
import glob
import json
import os
import re
import sqlite3
import sys


def short(name):
    """rocprof kernel name -> the HIP-event scope name bench.py reports
    (das_internal.h ProfScope): namespaces and the parameter list dropped,
    template arguments kept with unsigned int / long spelled u32 / u64, no
    spaces, e.g. "k_dj_write<2,1,u32>", "k_radix_scatter_lds<u64,true>"."""
    n = name.replace("das::(anonymous namespace)::", "").replace("das::", "").replace("void ", "")
    n = n.split("(", 1)[0]
    for a, b in (("unsigned long long", "u64"), ("unsigned long", "u64"), ("unsigned int", "u32"),
                 ("unsigned char", "u8")):
        n = n.replace(a, b)
    return n.replace(" ", "")


# kernels whose reads are dominated by isolated random loads (x1): probes,
# and the build's gathers through a permutation or a representative index
# (k_fill_atoms reads two 16-byte digests at rep[id], k_fill_targets the ids
# of each child, k_temp_type / k_apply_perm / k_remap_local 4-byte gathers)
RANDOM = {"k_tile_count<BitsPred>", "k_ij_mid", "k_bits_probe", "k_ij_lc", "k_ij_small", "k_anti_ij", "k_hset_insert",
          "k_hset_first", "k_hset_anti", "k_lookup", "k_lookup_pub",
          "k_fill_atoms", "k_fill_targets", "k_temp_type", "k_apply_perm", "k_remap_local", "k_gather_u32",
          "k_gather_u64", "k_scatter_pairs", "k_run_bucket"}


def fetch_factor(kernel):
    # the filtered expansion's walk (flag pass <0>, one-walk <2>, staged): one random
    # bitmap probe per output
    return 1.0 if kernel in RANDOM or kernel.startswith(("k_dj_filt<0,", "k_dj_filt<2,", "k_dj_filt_staged<")) else 2.0


def _last_counts():
    """LAST_FROM=<bench.json> (the build bench: one timed build after a small
    warm-up build): kernel -> its launch count in the timed region, so only
    the last that many dispatches of each kernel are averaged."""
    path = os.environ.get("LAST_FROM")
    if not path:
        return None
    with open(path) as f:
        line = [l for l in f if l.startswith("{")][-1]
    rec = json.loads(line)
    det = rec.get("detail")          # the compact last line names the full record
    if det:
        p = det if os.path.isabs(det) else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), det)
        if os.path.exists(p):
            with open(p) as f:
                rec = json.load(f)
    return {k: v["launches"] for k, v in rec.get("kernels", {}).items()}


def per_kernel(db_dir, counter):
    dbs = glob.glob(os.path.join(db_dir, "**", "*.db"), recursive=True)
    out = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, v, d in c.execute("select kernel_name, value, dispatch_id from counters_collection "
                                    "where counter_name = ?", (counter,)):
            out.setdefault(short(name), []).append((int(d), float(v) * 1024.0))
    k = int(os.environ.get("TOPK", "0"))
    last = _last_counts()
    res = {}
    for s, dv in out.items():
        v = [x[1] for x in sorted(dv)]                      # dispatch order
        if last is not None and last.get(s):
            v = v[-last[s]:]
        elif k:
            v = sorted(v)[-k:]
        res[s] = (sum(v), len(v))
    return res


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        fb, fn = fetch.get(k, (0.0, 0))
        wb, wn = write.get(k, (0.0, 0))
        if not fn or not wn:
            continue
        f = fetch_factor(k)
        rd = f * fb / fn
        wr = wb / wn
        res[k] = {"bytes_per_launch": rd + wr, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                  "fetch_size_raw_per_launch": fb / fn, "fetch_factor": f,
                  "launches_fetch_pass": fn, "launches_write_pass": wn,
                  "note": f"read = {f:g} x FETCH_SIZE ({'random probes' if f == 1 else 'streaming'}), "
                          "write = WRITE_SIZE; mean over "
                          + ("the timed build's launches (the last dispatches)" if os.environ.get("LAST_FROM")
                             else f"the {os.environ['TOPK']} largest launches" if os.environ.get("TOPK")
                             else "all launches")}
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
