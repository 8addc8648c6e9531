"""Does a sustained one-stream run of cfg2 launches slow down after a few ms
(NOT product code)?  rocprofv3 traces of `bench.py --streams 1 --steps 200`
show launches at 15.7-16.0 us for the first ~2 ms and 17-19 us after
(profiles/r5_cfg2_1s_prof_summary.txt).  This times windows of 50
consecutive launches with HIP events over long runs of
  flat:  the flat streaming read of the same 98.3 MB (scripts/probe_stream.hip)
  cs1:   the product kernel on one stream
  cs1_bpc16: the same with round 4's 16-blocks-per-CU grid
  rowsg: the product's row access pattern without descriptors or arithmetic
  cs2:   the product kernel on two streams
  burst: the product kernel, 20-launch bursts after 5 ms of idle
each phase after 100 ms of idle; one-stream phases read the shader clock
(s_memtime against s_memrealtime) between the two halves of every window.
One JSON line per phase."""
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch  # first: one HIP runtime per process

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import MODE_VALIDATE, Device  # noqa: E402

so = "/tmp/probe_sustain.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_stream.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p]
L.probe_rowsg_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
L.probe_clock_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
dev = Device(0)
os.environ["WGCS_BLOCKS_PER_CU"] = "16"
dev16 = Device(0)  # round 4's grid: 16 blocks per CU, grid-stride
del os.environ["WGCS_BLOCKS_PER_CU"]
torch.cuda.set_device(0)
n = 65536
arena_np, pkts_np, _ = synth.make_batch(n, 1500, kinds="tcp4", seed=synth.SEED)
nbytes = int(pkts_np["len"].astype(np.int64).sum())
R = 4
arenas = [torch.from_numpy(arena_np).to("cuda") for _ in range(R)]
pkts = torch.from_numpy(pkts_np.view(np.uint8)).to("cuda")
outs = [torch.empty(n * 2, dtype=torch.uint8, device="cuda") for _ in range(R)]
pout = [torch.empty(65536 * 256, dtype=torch.int32, device="cuda") for _ in range(2)]
strm = [torch.cuda.Stream(), torch.cuda.Stream()]
N = int(os.environ.get("SUSTAIN_LAUNCHES", "1000"))
W = 50
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(strm[0])
e1.record(strm[0])
torch.cuda.synchronize()


clk = torch.zeros(2 * (N // W + 1), dtype=torch.int64, device="cuda")


def window(k0, launch, slot, sync=True):
    """W launches (launch(k, m) enqueues launches k .. k+m-1 on stream 0) with
    the clock probe after the first half; GPU us per launch, probe excluded
    (sync=False: returns the events, read after the whole run)."""
    a, b, c, d = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    a.record(strm[0])
    launch(k0, W // 2)
    b.record(strm[0])
    L.probe_clock_launch(clk[2 * slot:].data_ptr(), strm[0].cuda_stream)
    c.record(strm[0])
    launch(k0 + W // 2, W - W // 2)
    d.record(strm[0])
    if not sync:
        return a, b, c, d
    torch.cuda.synchronize()
    return (a.elapsed_time(b) + c.elapsed_time(d)) * 1e3 / W


def cs_launcher(dv):
    lists = {}

    def go(k, m):  # one library call per half window (no per-launch Python)
        key = (k % R, m)
        if key not in lists:
            lists[key] = dv.batch_list([(arenas[(k + j) % R], pkts, n, outs[(k + j) % R]) for j in range(m)])
        dv.checksum_batches(MODE_VALIDATE, lists[key], strm[:1])
    return go


def flat(k, m):
    for j in range(k, k + m):
        L.probe_launch(arenas[j % R].data_ptr(), nbytes, pout[0].data_ptr(), 4096, 4, 1, strm[0].cuda_stream)


def rowsg(k, m):  # the product's G = 32, U = 4 row pattern on 1500-B slots, one pass, no descriptors or arithmetic
    for j in range(k, k + m):
        L.probe_rowsg_launch(arenas[j % R].data_ptr(), pkts.data_ptr(), n, 1500, pout[0].data_ptr(), n // 8, 32, 4, 0,
                             strm[0].cuda_stream)


def window_cs(k0, ns):
    bl = dev.batch_list([(arenas[(k0 + k) % R], pkts, n, outs[(k0 + k) % R]) for k in range(W)])
    dev.checksum_batches(MODE_VALIDATE, bl, strm[:ns], e0, e1)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / W


def report(phase, us, with_clock=True):
    r = {"phase": phase, "launches_per_window": W, "us_per_launch": [round(u, 2) for u in us],
         "frac_of_8TBps": [round(nbytes / u / 1e3 / 8000, 4) for u in us]}
    if with_clock:
        c = clk.cpu().numpy()
        r["sclk_mhz"] = [round(100.0 * c[2 * i] / max(c[2 * i + 1], 1)) for i in range(len(us))]
    print(json.dumps(r), flush=True)


AB = os.environ.get("SUSTAIN_AB")  # "a=K1:V1+K2:V2;b=..." -- launch-shape variants interleaved window by window
if AB:
    devs = {}
    for spec in AB.split(";"):
        name, _, kv = spec.partition("=")
        saved = dict(os.environ)
        for item in filter(None, kv.split("+")):
            k, _, v = item.partition(":")
            os.environ[k] = v
        devs[name] = cs_launcher(Device(0))
        os.environ.clear()
        os.environ.update(saved)
    for f in devs.values():
        window(0, f, 0)
    time.sleep(0.1)
    res = {name: ([], []) for name in devs}
    rounds = int(os.environ.get("SUSTAIN_ROUNDS", "20"))
    if os.environ.get("SUSTAIN_ASYNC"):  # every window enqueued back to back: no idle between them
        clk2 = torch.zeros(2 * rounds * len(devs), dtype=torch.int64, device="cuda")
        clk_saved, clk = clk, clk2
        evs = []
        for rnd in range(rounds):
            for i, (name, f) in enumerate(devs.items()):
                evs.append((name, window(rnd * W, f, rnd * len(devs) + i, sync=False)))
        torch.cuda.synchronize()
        c = clk.cpu().numpy()
        for j, (name, (a, b, cc, d)) in enumerate(evs):
            res[name][0].append(round((a.elapsed_time(b) + cc.elapsed_time(d)) * 1e3 / W, 2))
            res[name][1].append(round(100.0 * c[2 * j] / max(c[2 * j + 1], 1)))
        rounds = 0
    for rnd in range(rounds):
        for i, (name, f) in enumerate(devs.items()):
            clk.zero_()
            res[name][0].append(round(window(rnd * W, f, 0), 2))
            c = clk.cpu().numpy()
            res[name][1].append(round(100.0 * c[0] / max(c[1], 1)))
    for name, (us, mhz) in res.items():
        print(json.dumps({"variant": name, "async": bool(os.environ.get("SUSTAIN_ASYNC")), "spec": dict(x.split("=", 1) for x in AB.split(";"))[name],
                          "us_per_launch": us, "sclk_mhz": mhz}), flush=True)
    sys.exit(0)
LAUNCH = {"flat": flat, "cs1": cs_launcher(dev), "cs1_bpc16": cs_launcher(dev16), "rowsg": rowsg}
for f in LAUNCH.values():  # compile / first-use costs outside the phases
    window(0, f, 0)
for phase in os.environ.get("SUSTAIN_PHASES", "flat,cs1,rowsg,cs1_bpc16,cs2,burst,cs1").split(","):
    time.sleep(0.1)
    if phase in LAUNCH:
        clk.zero_()
        report(phase, [window(k, LAUNCH[phase], k // W) for k in range(0, N, W)])
    elif phase == "cs2":
        report(phase, [window_cs(k, 2) for k in range(0, N, W)], with_clock=False)
    elif phase == "burst":
        us = []
        for k in range(20):
            time.sleep(0.005)
            bl = dev.batch_list([(arenas[(k + j) % R], pkts, n, outs[(k + j) % R]) for j in range(20)])
            dev.checksum_batches(MODE_VALIDATE, bl, strm[:1], e0, e1)
            torch.cuda.synchronize()
            us.append(e0.elapsed_time(e1) * 1e3 / 20)
        print(json.dumps({"phase": phase, "launches_per_burst": 20, "idle_ms": 5,
                          "us_per_launch": [round(u, 2) for u in us]}), flush=True)
sys.exit(0)
