"""Cross-check of bench.py's roofline numbers against a rocprofv3 kernel trace of the same
command (VERDICT r3 ask 4).

The bench times `extend_only` (the RS launch pair) and `commit_only` (the NMT + DAH launches)
with HIP events on the SquareBatch's launch stream, over B squares at once. In the trace
those launches are the ones on that stream with the full-batch grids (the timed batch steps
split B into two chunks on two other streams, so their grids are half the size). This script
finds the stream of the full-batch rows launch, takes the median duration of every
(kernel, grid) on it (with batches in flight: after the other batches' last launch, i.e.
the phase timing alone), and rebuilds the line's `roofline.frac` and `roofline_nmt.achieved`.

usage: python tools/roofline_crosscheck.py <trace dir> <bench json> [k] [B]"""
import collections
import csv
import glob
import json
import statistics
import sys

SHA_MEASURED_PEAK = 29.4e9
# VALU instructions of one SHA-256 compression per wave, from the ISA of the unrolled
# compression (tools/microbench/sha_rate.hip k_sha_u, tools/isa_mix.py): alignbit, bitop3,
# add3, VOP2 (add / lshr / xor / mov)
SHA_ISA = {"v_alignbit_b32": 576, "v_bitop3_b32": 352, "v_add3_u32": 241, "vop2": 134 + 96 + 15}
# each op alone, dependency-free, 4 waves per SIMD, on the box of the sha_rate run
# (tools/microbench/vop3_banks.hip, profiles/r4_sha_ceiling.txt), lane-ops/s
SHA_OP_RATE = {"v_alignbit_b32": 32.15e12, "v_bitop3_b32": 57.0e12, "v_add3_u32": 32.3e12, "vop2": 61.0e12}


def main():
    tdir, bjson = sys.argv[1], sys.argv[2]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    rows = []
    for f in glob.glob(tdir + "/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    line = None
    for ln in open(bjson):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    nslice = 2  # 512-byte shares in 256-byte slices
    R = k * nslice * B // 4 * 256  # k axes of B squares: 4 tiles (waves) per 256-thread workgroup
    # the RS launch pair, by schedule (round 5: rows beside Q0 columns, then Q1 columns)
    pair_k = [r for r in rows if "k_rs_axis_gf8_pair" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 2 * R]
    if pair_k:
        first_name = pair_k[0]["Kernel_Name"]
        second_name = next(r["Kernel_Name"] for r in rows if "k_rs_axis_gf8<" in r["Kernel_Name"]
                           and int(r["Grid_Size_X"]) == R)
        launches = [(first_name, 2 * R, "rows + Q0 cols"), (second_name, R, "Q1 cols")]
    else:
        name = next(r["Kernel_Name"] for r in rows if "k_rs_axis_gf8" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == R)
        launches = [(name, R, "rows"), (name, 2 * R, "cols")]
    rs_names = {n for n, _, _ in launches}
    # the phase timing's stream: the one running most full-batch launches of the 2R-grid kernel
    big = [ln for ln in launches if ln[1] == 2 * R][0]
    bigc = [r for r in rows if r["Kernel_Name"] == big[0] and int(r["Grid_Size_X"]) == big[1]]
    stream = collections.Counter((r["Stream_Id"], r["Queue_Id"]) for r in bigc).most_common(1)[0][0]
    cand = [r for r in bigc if (r["Stream_Id"], r["Queue_Id"]) == stream]
    # the k-run's window: from its first full-batch RS launch to the first launch of
    # another RS kernel (the next shape's run: the k=512 line or a rider) after it
    t0 = min(int(r["Start_Timestamp"]) for r in cand)
    later = [int(r["Start_Timestamp"]) for r in rows if int(r["Start_Timestamp"]) > t0
             and ("k_rs" in r["Kernel_Name"] and r["Kernel_Name"] not in rs_names)]
    t1 = min(later) if later else float("inf")
    # --inflight > 1: the timed steps run full-batch launches on every batch's stream, two
    # batches at once; the phase timing (one batch alone) starts after the last of the
    # other batches' launches
    others = {(r["Stream_Id"], r["Queue_Id"]) for r in bigc} - {stream}
    ends = [int(r["End_Timestamp"]) for r in rows if (r["Stream_Id"], r["Queue_Id"]) in others
            and t0 <= int(r["Start_Timestamp"]) < t1]
    if ends:
        t0 = max(ends)
    on = [r for r in rows if (r["Stream_Id"], r["Queue_Id"]) == stream and t0 <= int(r["Start_Timestamp"]) < t1]
    d = collections.defaultdict(list)
    for r in on:
        d[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    P = out.append
    P(f"# roofline cross-check: rocprofv3 --kernel-trace of `python3 bench.py` vs its JSON line")
    P(f"# trace: {tdir}; line: {bjson}; k={k}, B={B}; launch stream {stream[0]} (queue {stream[1]}),")
    P(f"# the stream of the phase timing's full-batch RS launches, from the first of them")
    P(f"# (with batches in flight: from the other batches' last launch) to the next")
    P(f"# shape's first RS launch ({(t1 - t0) / 1e6 if t1 != float('inf') else 0:.1f} ms); medians over the calls")
    P(f"{'kernel':70s} {'grid':>10s} {'calls':>5s} {'median_us':>10s}")
    for (n, g), v in sorted(d.items(), key=lambda x: -statistics.median(x[1])):
        P(f"{n[:70]:70s} {g:10d} {len(v):5d} {statistics.median(v):10.1f}")
    parts = [(what, statistics.median(d[(n, g)])) for n, g, what in launches]
    pair = sum(t for _, t in parts)
    alg = 2048 * k * k * B
    frac = alg / (pair * 1e-6) / 8e12
    P("")
    P(f"RS launch pair (" + " + ".join(f"{w} {t:.1f}" for w, t in parts) + f") = {pair:.1f} us; algorithmic "
      f"2048 k^2 B = {alg / 1e9:.3f} GB -> {alg / pair / 1e3:.0f} GB/s = frac {frac:.4f} of 8 TB/s")
    nmt_keys = [(n, g) for (n, g) in d if any(s in n for s in ("k_leaf", "k_level", "k_merkle", "k_dah"))]
    # commit_only runs every NMT kernel once per call at the full-batch grids on this stream
    nmt = sum(statistics.median(d[key]) for key in nmt_keys)
    comp = (60 * k * k + 4 * k - 2) * B
    P(f"NMT + DAH launches ({len(nmt_keys)} kernels: " + ", ".join(f"{n.split('(')[0][-28:]}@{g}" for n, g in sorted(nmt_keys)) + ")")
    P(f"  sum of medians {nmt:.1f} us; {comp / 1e6:.1f} M compressions -> {comp / nmt / 1e3:.2f} G/s "
      f"= {comp / nmt / 1e3 / (SHA_MEASURED_PEAK / 1e9):.3f} of the measured SHA-256 peak")
    if line:
        rf, rn = line.get("roofline", {}), line.get("roofline_nmt", {})
        P("")
        P(f"bench line: roofline.avg_launch_us {rf.get('avg_launch_us', 0):.1f} (frac {rf.get('frac', 0):.4f}); "
          f"trace/line pair time {pair / rf.get('avg_launch_us', 1):.3f}")
        P(f"bench line: roofline_nmt.avg_launch_us {rn.get('avg_launch_us', 0):.1f} (achieved "
          f"{rn.get('achieved', 0):.2f} G/s); trace/line NMT time {nmt / rn.get('avg_launch_us', 1):.3f} "
          f"(trace = profiled run)")
    # SHA-256 ceilings for the NMT phase, three ways
    n_valu = sum(SHA_ISA.values())
    guide = 1024 * 2.4e9 * 64 / (2 * n_valu)
    model = 1.0 / sum(SHA_ISA[k] / SHA_OP_RATE[k] for k in SHA_ISA)
    rate = comp / nmt * 1e6
    P("")
    P(f"SHA-256 ceilings ({n_valu} VALU per compression per wave: " + ", ".join(f"{k} {v}" for k, v in SHA_ISA.items()) + ")")
    P(f"  MI355X_MICROARCH.md issue model (every wave64 VALU instruction over 2 cycles, 1024 SIMDs, 2.4 GHz): "
      f"{guide / 1e9:.1f} G/s -> NMT phase frac {rate / guide:.3f}")
    P(f"  the mix at each op's dependency-free rate on the compression's box (lane-ops/s: alignbit 32.15T, add3 "
      f"32.3T, bitop3 57.0T, VOP2 61.0T; profiles/r4_sha_ceiling.txt): {model / 1e9:.1f} G/s -> frac {rate / model:.3f}")
    P(f"  the same compression chained in registers, no memory traffic (profiles/r2_sha_rate.txt): "
      f"{SHA_MEASURED_PEAK / 1e9:.1f} G/s -> frac {rate / SHA_MEASURED_PEAK:.3f}")
    print("\n".join(out))


if __name__ == "__main__":
    main()
