"""Establish what aborts ProcessGroupNCCL's watchdog during a hipGraph capture.

Each case runs in its own child process (one rank, nccl process group, 1 GPU) because the
failure is a SIGABRT thrown from the watchdog thread:

  A  eager async all-reduce (its Work on the watchdog's list), then a capture in which an async
     all-reduce makes the process group's internal RCCL stream join the graph, held open 0.5 s
     so that a watchdog poll lands inside it; nothing retired before the capture
  B  as A, with graph_step.retire_collectives() before the capture
  C  as A, but the captured all-reduce is synchronous (it runs on the capture stream; the
     internal RCCL stream never joins the capture)
  D  graph_step.CapturedStep on a step that issues an async all-reduce and holds the capture
     open 0.3 s (its warm-up steps leave Works on the watchdog's list): the regression case of
     tests/test_distributed.py::test_captured_step_survives_watchdog_polls

    python tools/watchdog_capture_probe.py            # runs A, B, C, D; one summary line each
"""
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(case):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    from gasfm_amd.graph_step import retire_collectives
    os.environ.update(MASTER_ADDR="127.0.0.1", RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    x = torch.ones(1 << 20, device=dev)
    if case == "D":
        from gasfm_amd.graph_step import CapturedStep

        def fn():
            y = x * 2
            w2 = dist.all_reduce(y, async_op=True)
            time.sleep(0.3)
            w2.wait()
            return y.sum()
        step = CapturedStep(fn, [], warmup=2)
        v = float(step())
        print(f"case D: captured {step.captured} ({step.fallback_reason}), loss {v}", flush=True)
        assert step.captured and v == 2.0 * x.numel()
        dist.destroy_process_group()
        return
    w = dist.all_reduce(x, async_op=True)  # listed on the watchdog until a poll sees it complete
    w.wait()
    torch.cuda.synchronize()
    if case == "B":
        retire_collectives()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        y = x * 2
        if case == "C":
            dist.all_reduce(y)
        else:
            w2 = dist.all_reduce(y, async_op=True)
        time.sleep(0.5)  # >= 4 watchdog polls while the capture (and in A/B the RCCL stream) is open
        if case != "C":
            w2.wait()
        z = y + 1
    g.replay()
    torch.cuda.synchronize()
    ok = bool((z == 3).all())
    print(f"case {case}: replayed, values {'ok' if ok else 'WRONG'}", flush=True)
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    for case in sys.argv[1:] or ("A", "B", "C", "D"):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29600 + ord(case)))
        t0 = time.time()
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", case], env=env,
                           capture_output=True, text=True, timeout=120)
        with open(os.path.join(REPO, "gpurun_out", f"watchdog_probe_{case}.log"), "w") as f:
            f.write(r.stdout + "\n---- stderr\n" + r.stderr)
        why = [ln.strip() for ln in r.stderr.splitlines()
               if "terminated with exception" in ln or "HIP error" in ln or "hipError" in ln][:3]
        print(f"case {case}: rc {r.returncode} in {time.time() - t0:.1f}s; {r.stdout.strip()} "
              f"{' | '.join(why)}", flush=True)


if __name__ == "__main__":
    main()
