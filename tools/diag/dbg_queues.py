"""Diagnostic: which stream pairs of a process run concurrently (distinct hardware queues).

Two spin kernels (torch.cuda._sleep, one thread each) on streams A and B: ~T when the
streams sit on different hardware queues, ~2T when they share one.  Stream kinds:
  null        the default (legacy) stream
  pool[i]     torch pool streams, in creation order
  hi[i]       high-priority pool streams
  cumask[i]   hipExtStreamCreateWithCUMask with every CU enabled
  plain[i]    hipStreamCreateWithFlags(NonBlocking)
    python tools/diag/dbg_queues.py [--pg]     (--pg: a one-rank RCCL group first)
"""
import ctypes as C
import os
import sys
import time

import torch


def hip():
    return C.CDLL("libamdhip64.so")


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if "--pg" in sys.argv:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29577")
        import torch.distributed as dist
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        t = torch.ones(4, device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
    h = hip()
    streams = {"null": torch.cuda.default_stream(dev)}
    for i in range(5):
        streams[f"pool{i}"] = torch.cuda.Stream(device=dev)
    for i in range(3):
        streams[f"hi{i}"] = torch.cuda.Stream(device=dev, priority=-1)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ncu + 31) // 32
    mask = (C.c_uint32 * words)(*([0xFFFFFFFF] * words))
    for i in range(3):
        s = C.c_void_p()
        rc = h.hipExtStreamCreateWithCUMask(C.byref(s), C.c_uint32(words), mask)
        if rc == 0:
            streams[f"cumask{i}"] = torch.cuda.ExternalStream(s.value, device=dev)
        else:
            print("hipExtStreamCreateWithCUMask rc", rc)
    for i in range(3):
        s = C.c_void_p()
        rc = h.hipStreamCreateWithFlags(C.byref(s), C.c_uint(1))
        if rc == 0:
            streams[f"plain{i}"] = torch.cuda.ExternalStream(s.value, device=dev)
    cyc = 2_000_000
    main_st = torch.cuda.current_stream(dev)

    def run(names):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_st)
        for nm in names:
            st = streams[nm]
            st.wait_event(e0)
            with torch.cuda.stream(st):
                torch.cuda._sleep(cyc)
        for nm in names:
            main_st.wait_stream(streams[nm])
        e1.record(main_st)
        e1.synchronize()
        return e0.elapsed_time(e1)
    one = min(run(["pool0"]) for _ in range(3))
    cyc = max(1000, int(cyc * 20.0 / max(one, 1e-3)))  # ~20 ms per spin
    one = min(run(["pool0"]) for _ in range(3))
    print(f"one spin: {one:.2f} ms  (streams: {', '.join(streams)})")
    names = list(streams)
    for i, a in enumerate(names):
        shared = []
        for b in names[i + 1:]:
            t = min(run([a, b]) for _ in range(2))
            if t > 1.5 * one:
                shared.append(b)
        print(f"{a:8s} shares a queue with: {', '.join(shared) if shared else '-'}", flush=True)


if __name__ == "__main__":
    main()
