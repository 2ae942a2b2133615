"""Hashed multi-key group-by (option no_pack) with many groups, so that it
takes the partitioned path with large partition tables: exact vs pandas,
and (under the checked library, PLGPU_LIB=.../libpolaroid_gpu_checked.so)
the index-invariant bits of plgpu_debug_checks.

    PLGPU_LIB=polaroid_amd/libpolaroid_gpu_checked.so python tools/diag_hashed_partitioned.py [--groups 700000]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--groups", type=int, default=700_000)
    args = ap.parse_args()
    import pandas as pd

    import polaroid_amd as pl
    from polaroid_amd import _native as N

    N.set_option("no_pack", 1)
    rng = np.random.default_rng(99)
    n = args.rows
    side = int(np.sqrt(args.groups)) + 1
    k1 = rng.integers(0, side, n).astype(np.int64)
    k2 = rng.integers(0, side, n).astype(np.int64)
    a = rng.standard_normal(n)
    b = rng.integers(-9, 9, n).astype(np.int64)
    df = pl.DataFrame({"k1": pl.Series.from_numpy("k1", k1), "k2": pl.Series.from_numpy("k2", k2),
                       "a": pl.Series.from_numpy("a", a), "b": pl.Series.from_numpy("b", b)})
    info = {}
    try:
        out = df.lazy().group_by("k1", "k2").agg(pl.col("a").sum(), pl.col("b").max(), pl.len()).collect(info=info)
    except Exception as e:  # noqa: BLE001
        bits = C.c_uint32(0)
        rc = N.lib().plgpu_debug_checks(C.byref(bits))
        print(json.dumps({"error": str(e), "debug_checks_rc": rc, "check_bits": bits.value}), flush=True)
        return
    bits = C.c_uint32(0)
    rc = N.lib().plgpu_debug_checks(C.byref(bits))
    ref = pd.DataFrame({"k1": k1, "k2": k2, "a": a, "b": b}).groupby(["k1", "k2"]).agg(
        b=("b", "max"), len=("a", "size")).reset_index()
    got = pd.DataFrame({"k1": out["k1"].to_numpy(), "k2": out["k2"].to_numpy(), "b": out["b"].to_numpy(),
                        "len": out["len"].to_numpy()})
    m = ref.merge(got, on=["k1", "k2"], suffixes=("_r", "_g"), how="outer", indicator=True)
    ok = bool((m["_merge"] == "both").all() and (m["b_r"] == m["b_g"]).all() and (m["len_r"] == m["len_g"]).all())
    print(json.dumps({"groups": out.height, "ref_groups": len(ref), "match": ok, "debug_checks_rc": rc,
                      "check_bits": bits.value, "path": info.get("path"), "reruns": info.get("reruns")}), flush=True)


if __name__ == "__main__":
    main()
