"""Host codec throughput (codecs.go:15-27 / 84-93) on the c3 input:
1M partitions x 1000 brokers, 64-broker allowed lists, Zipf weights, as JSON.

Times the CLI's decode (one-pass decoder, the partitions array split over up to 16
threads at chunk boundaries it proves; DOM fallback never taken on this input) and the Go-compatible encode of the whole list (contiguous slices on up
to 16 threads), in MB/s of JSON;
the DOM parser + decoder (the pre-fast-path implementation, a node per value) is
timed on a 100k-partition slice for comparison.  Byte parity of the encoder with
the oracle's writer is tests/test_codec.py's job.  Prints one JSON line.

Usage: python tools/codec_bench.py [--partitions N] [--out profiles/...json]
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kafkabalancer_amd import cli, synth  # noqa: E402


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--partitions", type=int, default=1_000_000)
    ap.add_argument("--dom-partitions", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    t0 = time.perf_counter()
    cl, cfg, desc = synth.config("c3", scale=a.partitions / 1_000_000)
    cl.topics = None
    pl = synth.to_plist(cl)
    data = json.dumps(pl, separators=(",", ":")).encode()
    n_dom = min(a.dom_partitions, len(pl["partitions"]))
    dom_data = json.dumps({"version": 1, "partitions": pl["partitions"][:n_dom]}, separators=(",", ":")).encode()
    del pl
    gen_s = time.perf_counter() - t0
    mb = len(data) / 1e6
    best_p = best_e = None
    out_mb = 0.0
    for _ in range(a.reps):
        rc, out, tp, te, n = cli.codec_roundtrip(data, cli.CODEC_DEFAULT)
        assert rc == 0 and n == cl.n, out[:200]
        out_mb = len(out) / 1e6
        del out
        best_p = tp if best_p is None else min(best_p, tp)
        best_e = te if best_e is None else min(best_e, te)
    fast_only = cli.codec_roundtrip(dom_data, cli.CODEC_FAST)[0] == 0
    rc, _, tp_dom, te_dom, _ = cli.codec_roundtrip(dom_data, cli.CODEC_DOM)
    assert rc == 0
    rc, _, tp_fast_slice, _, _ = cli.codec_roundtrip(dom_data, cli.CODEC_DEFAULT)
    res = {
        "what": "host codec throughput, c3 JSON (SURVEY.md 8(f1); codecs.go:15-27 decode, :84-93 encode)",
        "input": {"partitions": cl.n, "brokers": 1000, "allowed_list": 64, "weights": "zipf",
                  "json_mb": round(mb, 1), "generated_s": round(gen_s, 1)},
        "decode": {"s": round(best_p, 3), "mb_per_s": round(mb / best_p, 1),
                   "path": "one-pass decoder (no DOM fallback on this input: %s)" % fast_only},
        "encode": {"s": round(best_e, 3), "mb_per_s": round(out_mb / best_e, 1), "out_mb": round(out_mb, 1)},
        "dom_baseline": {"partitions": n_dom, "decode_mb_per_s": round(len(dom_data) / 1e6 / tp_dom, 1),
                         "one_pass_decode_mb_per_s_same_slice": round(len(dom_data) / 1e6 / tp_fast_slice, 1),
                         "note": "DOM parser + decoder (a node per JSON value), the pre-fast-path CLI"},
        "decode_threads": int(os.environ.get("KB_CODEC_THREADS", "0")) or
                          (min(16, os.cpu_count() or 1) if len(data) >= (8 << 20) else 1),
        "encode_threads": int(os.environ.get("KB_CODEC_THREADS", "0")) or min(16, os.cpu_count() or 1),
        "cpu_model": cpu_model(), "nproc": os.cpu_count(), "reps": a.reps,
        "reference": "Go encoding/json is not buildable here (no Go toolchain); no reference timing",
    }
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
