#!/usr/bin/env python3
"""Summarises the mirrored pipeline's per-chunk timelines (RSAMD_TRACE of the
TUNING build, host.cpp MirrorTrace; tools/host_legs.py --trace writes them):
per call, where the wall time goes -- the fill (call start to the first
kernel), the kernels' busy time, the gaps between one chunk's kernel end and
the next one's start (and what the host was doing then), and the drain (last
kernel end to the call's end).  Times in microseconds.
  python tools/mirror_trace.py TRACE.jsonl"""
import json
import sys


def summarise(call):
    ch = call["chunks"]
    us = lambda ns: round(ns / 1e3, 1)  # noqa: E731
    ks = [c["kernel"][0] for c in ch]
    ke = [c["kernel"][1] for c in ch]
    busy = sum(e - s for s, e in zip(ks, ke))
    gaps = [ks[j + 1] - ke[j] for j in range(len(ch) - 1)]
    # a gap's cause: the next chunk's kernel was launched after the previous
    # one ended (the host was still copying its inputs) or not
    late = [ch[j + 1]["launch"] - ke[j] for j in range(len(ch) - 1)]
    return {
        "bytes": call["bytes"], "chunks": len(ch), "total_us": us(call["total_ns"]),
        "fill_us": us(ks[0]), "kernel_busy_us": us(busy), "drain_us": us(call["total_ns"] - ke[-1]),
        "gaps_us": [us(g) for g in gaps], "launch_after_prev_end_us": [us(x) for x in late],
        "copy_us": [us(c["copy"][1] - c["copy"][0]) for c in ch],
        "kernel_us": [us(e - s) for s, e in zip(ks, ke)],
    }


def main():
    for line in open(sys.argv[1]):
        line = line.strip()
        if line.startswith("{"):
            print(json.dumps(summarise(json.loads(line))))


if __name__ == "__main__":
    main()
