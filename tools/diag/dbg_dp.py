"""Diagnostic: the two micro-batch engine streams and the hardware queues they land on.

HIP maps every stream of a process onto one of GPU_MAX_HW_QUEUES (4) hardware queues
per priority; two engine streams on the same queue run one after the other.  Each
variant runs in a FRESH child process (stream creation order decides the queues):
    python tools/dbg_dp.py [steps]
variant = mode (plain | staged | reducer: DP at one rank) x the engine-1 stream's
priority (0: normal, as engine 0's default stream; -1: high) x extra pool streams taken
before the trainer (shifts which queue engine 1 lands on).
"""
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def child(mode, prio, pre, steps):
    sys.path.insert(0, os.path.join(HERE, "..", "..", "super-resolution-climate_amd"))
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import torch
    from srmi.dist import init_from_env
    from srmi.engine import NetSpec
    from srmi.trainer import FusedTrainer
    import bench
    info = init_from_env(None, force=(mode != "plain"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    keep = [torch.cuda.Stream(device=dev) for _ in range(pre)]
    orig = torch.cuda.Stream
    if prio:
        torch.cuda.Stream = lambda device=None, priority=0, **kw: orig(device=device, priority=prio, **kw)
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4)
    tr = FusedTrainer(spec, 64, (48, 48), lr=1e-4, info=info, device=dev, seed=0, micro=2,
                      dp_reducer_stream=(mode == "reducer"))
    torch.cuda.Stream = orig
    hr = torch.tensor(bench.synthetic_hr(64, 2, 192, 1234)).to(dev)
    for _ in range(4):
        tr.step(hr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = tr.step(hr)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"RESULT {mode:8s} prio {prio:2d} pre {pre}: {1000 * dt:8.3f} ms/step {64 / dt:8.1f} tiles/s "
          f"loss {float(out['loss']):.6f}", flush=True)
    del keep


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
        sys.exit(0)
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    port = 29600
    for mode in ("plain", "staged", "reducer"):
        for prio in (0, -1):
            for pre in (0, 1, 2, 3):
                port += 1
                env["MASTER_PORT"] = str(port)
                r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode, str(prio), str(pre),
                                    str(steps)], env=env, capture_output=True, text=True, timeout=180)
                line = [x for x in r.stdout.splitlines() if x.startswith("RESULT")]
                print(line[0] if line else f"{mode} {prio} {pre}: failed rc={r.returncode} {r.stderr[-300:]}",
                      flush=True)
                if r.returncode != 0:
                    sys.exit(1)
