#!/usr/bin/env python3
"""Where k_pieces' extra HBM reads on C5 come from: a CPU model of the launch's read
REQUESTS (not its CRCs).  Mirrors csrc/crc32_kernels.hip k_pieces + WaveSplit +
pieces_loop: 256 workgroups x 16 waves, wave ranges balanced by pieces, the round cut
at the first window outside the slot span, the speculative span prefetch (hit / miss
reload) and the per-round metadata loads.  Counts, per launch, the 128-B lines each
source requests, how many of them were already requested earlier by the same wave
(the span overlap between consecutive rounds), by the previous wave (range
boundaries), and the unique footprint.  FETCH_SIZE (x2) on the GPU then says how many
of the repeated requests missed L2.  TEST/MEASUREMENT INFRASTRUCTURE, not the product.

    python tools/c5_span_model.py [--n 1048576] [--s 1.1] [--out profiles/r05/c5_span_model.json]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

S = 64                      # kPieceS
CHUNKS = 272                # kPcChunks: span chunks a slot holds
SPAN = 16 * CHUNKS          # kSpanBytes
POS = 290                   # kPcSlotPos: DMA positions (every 17th a duplicate chunk)
DMA_CHUNKS = [q - q // 17 for q in range(POS)]
LINE = 128


def dma_lines(b16: int, lim: int | None = None) -> set:
    """128-B lines the 5 LDS-DMA instructions of one span request; with lim, the lanes
    whose chunk starts at or past byte lim are left out (tail clamp)."""
    return {(b16 + 16 * c) // LINE for c in set(DMA_CHUNKS) if lim is None or b16 + 16 * c < lim}


def model(offs, lens, grid=256, waves=16, chunks=CHUNKS, spec_back=S, clamp=False):
    """clamp: the prefetch of a round whose view holds every packet the wave has left
    stops at the end of the last of them (WTP_PC_TAILCLAMP)."""
    n = len(lens)
    k_all = np.where((lens == 0) | (lens > 4096), 1, (lens + S - 1) // S).astype(np.int64)
    tw = grid * waves
    st = {"span_line_requests": 0, "span_lines_seen_by_wave": 0, "span_lines_seen_by_prev_wave": 0,
          "miss_reloads": 0, "rounds": 0, "meta_line_requests": 0, "meta_lines_seen_by_wave": 0,
          "consumed_span_bytes": 0, "span_bytes_issued": 0}
    span_seen_global = set()
    prev_wave_lines = set()
    for g in range(grid):
        g0, g1 = n * g * waves // tw, n * (g + 1) * waves // tw
        if g0 == g1:
            continue
        kk = k_all[g0:g1]
        excl = np.concatenate([[0], np.cumsum(kk)[:-1]])
        total = int(kk.sum())
        starts = [g0] + [g0 + int(np.searchsorted(excl, (total * w) // waves, side="left")) for w in range(1, waves)] + [g1]
        for w in range(waves):
            lo, hi = starts[w], starts[w + 1]
            seen, mseen = set(), set()
            p0, skip, spec = lo, 0, None
            while p0 < hi:
                navail = min(64, hi - p0)
                ks = k_all[p0:p0 + navail].copy()
                ks[0] -= skip
                inc = np.cumsum(ks)
                covered = int(inc[-1])
                # lane -> (packet, piece) for the first min(64, covered) lanes
                lanes = []
                pk = 0
                for lane in range(min(64, covered)):
                    while inc[pk] <= lane:
                        pk += 1
                    lp = lane - (int(inc[pk]) - int(ks[pk]))
                    gp = lp + (skip if pk == 0 else 0)
                    K = int(k_all[p0 + pk])
                    we = int(offs[p0 + pk]) + int(lens[p0 + pk]) - (K - 1 - gp) * S
                    lanes.append((pk, gp, K, we - S, we))
                lo16 = lanes[0][3] & ~15
                tot = len(lanes)
                for i, (_, _, _, ws, we) in enumerate(lanes):
                    if ws < lo16 or we - lo16 > chunks * 16:
                        tot = i
                        break
                act = lanes[:tot]
                hit = spec is not None and all(ws >= spec and we - spec <= chunks * 16 for _, _, _, ws, we in act)
                if not hit:
                    st["miss_reloads"] += 1
                    L = dma_lines(lo16)
                    st["span_line_requests"] += len(L)
                    st["span_lines_seen_by_wave"] += len(L & seen)
                    st["span_lines_seen_by_prev_wave"] += len(L & prev_wave_lines)
                    seen |= L
                st["consumed_span_bytes"] += act[-1][4] - max(act[0][3], lo16)
                # metadata of the next round: lanes load packets p0n .. p0n+63 (clamped)
                pk_l, gp_l, K_l, _, we_l = act[-1]
                partial = gp_l + 1 < K_l
                p0n = p0 + pk_l + (0 if partial else 1)
                if p0n < hi:
                    ml = set()
                    for base, width in ((0, 8), (1 << 40, 4)):  # offsets (u64), lengths (u32)
                        a, b = p0n, min(p0n + 64, hi)
                        ml |= {(base + width * p) // LINE for p in (a, b - 1)} | \
                              {(base + width * p) // LINE for p in range(a, b, LINE // width)}
                    st["meta_line_requests"] += len(ml)
                    st["meta_lines_seen_by_wave"] += len(ml & mseen)
                    mseen |= ml
                spec = ((we_l - spec_back) & ~15) if p0n < hi else None
                if spec is not None:
                    lim = None
                    if clamp and hi - p0 <= 64:
                        lim = max(int(offs[q]) + int(lens[q]) for q in range(p0n, hi))
                    L = dma_lines(spec, lim)
                    st["span_line_requests"] += len(L)
                    st["span_lines_seen_by_wave"] += len(L & seen)
                    st["span_lines_seen_by_prev_wave"] += len(L & prev_wave_lines)
                    seen |= L
                st["span_bytes_issued"] += SPAN
                st["rounds"] += 1
                skip = gp_l + 1 if partial else 0
                p0 = p0n
            prev_wave_lines = seen
            span_seen_global |= seen
    st["span_unique_lines"] = len(span_seen_global)
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--s", type=float, default=1.1)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--out", default=None)
    ap.add_argument("--clamp", action="store_true", help="model the tail-clamped prefetch")
    a = ap.parse_args()
    lens = O.zipf_lengths(a.n, s=a.s).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    st = model(offs, lens, grid=a.grid, clamp=a.clamp)
    payload = int(lens.sum())
    algo = payload + 12 * a.n
    req = st["span_line_requests"] * LINE
    res = {"workload": f"C5: {a.n} packets, Zipf({a.s}) lengths 1..1456, packed", "tail_clamp": a.clamp,
           "payload_bytes": payload,
           "algorithmic_read_bytes": algo, "model": st,
           "span_request_bytes": req, "span_request_ratio_to_payload": round(req / payload, 4),
           "span_rerequest_bytes_same_wave": st["span_lines_seen_by_wave"] * LINE,
           "span_rerequest_bytes_prev_wave": st["span_lines_seen_by_prev_wave"] * LINE,
           "span_unique_bytes": st["span_unique_lines"] * LINE,
           "meta_request_bytes": st["meta_line_requests"] * LINE,
           "meta_rerequest_bytes_same_wave": st["meta_lines_seen_by_wave"] * LINE,
           "mean_consumed_span_bytes_per_round": round(st["consumed_span_bytes"] / st["rounds"], 1)}
    print(json.dumps(res, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
