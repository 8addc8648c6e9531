#!/usr/bin/env python3
"""Interleaved timing of GSO-kernel probe builds on cfg4 (round 2).

Each variant is the library built with timing-only -D switches that existed
only in the experimental revisions of gso_kernels.hip this script was run
against (wrong output by design, except `base`; the switches were removed
with the experiment, the outputs are kept in profiles/r2_probe_gso_*.jsonl):
  WGCS_P_NT=false    regular (temporal) payload loads instead of non-temporal
  WGCS_P_PLAINLD     first payload batch without ld_window's page-crossing test
  WGCS_P_PLAINST     full 16-byte stores for every payload chunk (no partial-chunk pieces)
  WGCS_P_OLDTAIL     the segment's last partial chunk as byte/short/dword pieces instead of one
                     full store merged with the slot's bytes read ahead
  WGCS_P_NTST        non-temporal payload stores
  WGCS_P_U=n         n payload windows per lane in flight (default 6; now the
                     product tunable WGCS_GSO_U)
  WGCS_P_NODEC       the decoder wave publishes the rows' own geometry instead
                     of decoding (no validation, zero header constants)
  WGCS_P_CONSTJOB    the rows take cfg4's job descriptor and virtio header as
                     constants (no dependent loads before the payload loads)
  WGCS_P_NOBAR       no decoder, no LDS barrier: the rows use their own geometry
  WGCS_P_WPE=n       amdgpu_waves_per_eu(n): VGPR budget for n waves per SIMD
                     (now the product tunable WGCS_GSO_WAVES, default 5)
  WGCS_P_BUF=0/1     payload windows through flat global loads (page test per
                     window) or raw buffer loads over the job's bytes (range check)
  WGCS_P_PRIO=n      s_setprio(n) once a row's payload loads are issued
  WGCS_P_DEADEXIT=1  segment groups past the job's last segment (bounded from
                     the virtio header alone) retire before the verdict
  WGCS_P_HBUF=1      the header chunks through raw buffer loads too
  WGCS_P_EARLY=0/1   first payload batch issued before (1) or after (0) the
                     data-offset check (the decoded path is an out-of-line call)
  WGCS_P_A16=0/1     payload windows dword-aligned (alignbyte + 1 DPP dword) or
                     16-byte aligned (funnel + 4 DPP dwords)
(An earlier run of this script timed a two-kernel design -- plan kernel +
segment kernel -- with switches that no longer exist; its output is
profiles/r2_probe_gso_plan_kernel.jsonl.)
Build on the CPU side first (`python scripts/probe_gso_variants.py build`),
then run on the GPU (`python scripts/probe_gso_variants.py [rounds]`): per
variant and round, GPU time per step from HIP events over K=200 launches on
one stream, and the same with two streams alternating.
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUTDIR = os.path.join(ROOT, "scripts", "probe_so")
VARIANTS = {
    "head": None,  # the committed kernel, built from `git archive HEAD` (see build())
    "store_dw": [],  # store_chunk pieces picked by dword selects (no 128-bit shifts)
}


def build():
    from wireguard_amd import build as B

    os.makedirs(OUTDIR, exist_ok=True)
    for k, defs in VARIANTS.items():
        out = os.path.join(OUTDIR, f"libwgcsum_{k}.so")
        if defs is None:  # HEAD's sources, unpacked by the caller into /tmp/headtree
            csrc = B.CSRC
            B.CSRC = "/tmp/headtree/wireguard_amd/csrc"
            try:
                B.build(out=out)
            finally:
                B.CSRC = csrc
        else:
            B.build(out=out, extra=[f"-D{d}" for d in defs])
        print("built", out, flush=True)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import numpy as np
    import torch

    from wireguard_amd import _lib, synth
    from wireguard_amd.tun import GSO_JOB_DTYPE, Device

    torch.cuda.set_device(0)
    devs = {}
    for k in VARIANTS:
        _lib._lib = None
        _lib.LIB_PATH = os.path.join(OUTDIR, f"libwgcsum_{k}.so")
        devs[k] = Device(0)
    n_jobs, total, gso, max_segs, stride, offset = 256, 65535, 1460, 64, 1536, 16
    max_segs = int(os.environ.get("WGCS_PROBE_MAX_SEGS", max_segs))  # output slots per job (45 used)
    pkts = [synth.make_super_packet(total, gso, seed=synth.SEED + k) for k in range(n_jobs)]
    jlen = len(pkts[0])
    arena = np.frombuffer(b"".join(pkts) + bytes(64), dtype=np.uint8).copy()
    jobs = np.zeros(n_jobs, GSO_JOB_DTYPE)
    jobs["off"] = np.arange(n_jobs, dtype=np.uint64) * np.uint64(jlen)
    jobs["len"] = jlen
    R = 8
    d_arena = [torch.from_numpy(arena).cuda() for _ in range(R)]
    d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
    d_out = [torch.empty(n_jobs * max_segs * stride, dtype=torch.uint8, device="cuda") for _ in range(R)]
    res = [[torch.zeros(n, dtype=torch.int32, device="cuda") for n in (n_jobs * max_segs, n_jobs, n_jobs)]
           for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bytes_step = int(jobs["len"].sum()) + 256 * (44 * 1500 + 1335)

    def run(dev, K, ns, k0=0):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(streams[0])
        if ns == 2:
            streams[1].wait_event(e0)
        for k in range(K):
            i, q = (k0 + k) % R, k % ns
            dev.gso_split_batch(d_arena[i], d_jobs, n_jobs, d_out[i], stride, offset, max_segs, res[q][0], res[q][1],
                                res[q][2], stream=streams[q])
        if ns == 2:
            j = torch.cuda.Event()
            j.record(streams[1])
            streams[0].wait_event(j)
        e1.record(streams[0])
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / K

    for k, d in devs.items():
        run(d, 20, 1)
    t = {k: {"s1": [], "s2": []} for k in VARIANTS}
    for _ in range(rounds):
        for k, d in devs.items():
            t[k]["s1"].append(run(d, 200, 1, 3))
            t[k]["s2"].append(run(d, 200, 2, 5))
    for k, v in t.items():
        o = {"variant": k, "defines": VARIANTS[k]}
        for m, xs in v.items():
            o[m + "_us_med"] = round(statistics.median(xs), 3)
            o[m + "_us_min"] = round(min(xs), 3)
            o[m + "_frac"] = round(bytes_step / (statistics.median(xs) * 1e-6) / 8e12, 4)
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        main()
