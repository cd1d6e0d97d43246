"""Do two HIP streams run concurrently?  torch.cuda._sleep (a one-block spin kernel) on two
streams: ~1x the spin time if they overlap, ~2x if they share a hardware queue.  Pairs: the
default stream with successive pool streams, with high-priority streams, and with streams
created by hipStreamCreate (ctypes)."""
import ctypes
import json
import time

import torch


def pair_ms(s1, s2, cycles=20_000_000):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s1):
        torch.cuda._sleep(cycles)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    torch.cuda.init()
    d = torch.cuda.current_stream()
    for _ in range(3):
        pair_ms(d, d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(20_000_000)
    torch.cuda.synchronize()
    one = (time.perf_counter() - t0) * 1e3
    out = {"one_spin_ms": round(one, 2), "pool": [], "high_prio": [], "hip_created": []}
    for i in range(8):
        s = torch.cuda.Stream()
        out["pool"].append(round(pair_ms(d, s) / one, 2))
    for i in range(4):
        s = torch.cuda.Stream(priority=-1)
        out["high_prio"].append(round(pair_ms(d, s) / one, 2))
    hip = ctypes.CDLL("libamdhip64.so")
    for i in range(6):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0  # non-blocking
        s = torch.cuda.ExternalStream(h.value)
        out["hip_created"].append(round(pair_ms(d, s) / one, 2))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
