#!/usr/bin/env python3
"""Batched Keccak-256 throughput (SURVEY.md §8a row A12, §8d "Keccak unit").

Messages are device-resident (mg_keccak256_device), one per lane; the digests
of a sample are checked against the oracle (oracle/keccak.py) first.
Algorithmic work: 7 248 u32 ops per 136-byte block (24 rounds x (theta 50 +
rho/pi 25 rotations + chi 75 + iota 1) u64 ops, x2 for 32-bit halves).
Writes gpurun_out/keccak_bench.json.
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OPS_PER_BLOCK = 7248


def main():
    import torch
    from mythril_amd.runtime import Device, MgStats, _check
    from oracle.keccak import keccak256

    dev = Device(0)
    res = {}
    peak = json.load(open(os.path.join(os.path.dirname(__file__), "..", "profiles", "valu_peak.json")))
    peak = float(peak["measured_ops_per_s"])
    for mlen, n in ((32, 1 << 22), (64, 1 << 22), (200, 1 << 21)):
        rng = np.random.default_rng(mlen)
        data = rng.integers(0, 256, size=n * mlen, dtype=np.uint8)
        offs = (np.arange(n, dtype=np.uint64) * mlen)
        lens = np.full(n, mlen, dtype=np.uint32)
        d_data = torch.from_numpy(data).cuda()
        d_off = torch.from_numpy(offs.view(np.int64)).cuda()
        d_len = torch.from_numpy(lens.view(np.int32)).cuda()
        d_out = torch.empty(32 * n, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        st = MgStats()
        for rep in range(4):
            _check(dev.lib, dev.lib.mg_keccak256_device(dev.handle, d_data.data_ptr(), d_off.data_ptr(),
                                                        d_len.data_ptr(), n, d_out.data_ptr(), ctypes.byref(st)),
                   "mg_keccak256_device")
        out = d_out.cpu().numpy()
        for i in list(range(8)) + [n - 1]:
            assert out[32 * i:32 * i + 32].tobytes() == keccak256(data[i * mlen:(i + 1) * mlen].tobytes()), i
        blocks = mlen // 136 + 1
        hs = n / (st.kernel_ms / 1e3)
        ach = hs * blocks * OPS_PER_BLOCK
        res[f"{mlen}B"] = {"messages": n, "blocks_per_msg": blocks, "kernel_ms": st.kernel_ms,
                           "hashes_per_s": hs, "u32_ops_per_s": ach, "frac_peak": ach / peak}
        print(f"{mlen:4d} B x {n}: {st.kernel_ms:.3f} ms, {hs / 1e9:.2f} G hashes/s, "
              f"{ach / 1e12:.2f} T u32-ops/s ({100 * ach / peak:.1f}% of measured peak)", flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/keccak_bench.json", "w"), indent=1)


if __name__ == "__main__":
    main()
