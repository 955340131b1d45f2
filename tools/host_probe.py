"""Host CPU facts of the GPU box for the CPU-baseline thread choice: os.cpu_count(), the affinity mask, the cgroup CPU
quota, and the CPU oracle's train step (n_feat=128, bs=8) at several thread counts."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cgroup_quota():
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(p).read().split()
            return None if q == "max" else float(q) / float(per)
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q < 0 else q / per
    except (OSError, ValueError):
        return None


def main():
    from oracle import ref_cpu as R
    aff = len(os.sched_getaffinity(0))
    print(f"os.cpu_count()={os.cpu_count()} affinity={aff} cgroup_quota={cgroup_quota()} "
          f"torch_default_threads={torch.get_num_threads()}", flush=True)
    nf, B, T = 128, 8, 1500
    torch.manual_seed(0)
    from cdm_amd.model import ContextUnet
    sd = R.clone_sd(ContextUnet(1, nf, 6, 64).state_dict())
    _, _, ab = R.make_schedule(T)
    g = torch.Generator().manual_seed(1)
    x = torch.rand(B, 1, 64, 64, generator=g); c = torch.rand(B, 6, generator=g)
    for th in sorted({8, 16, 32, aff, os.cpu_count()}):
        if th > 4 * aff:
            continue
        torch.set_num_threads(th)
        tr = R.OracleTrainer(sd, n_feat=nf, n_cfeat=6, height=64)
        noise = torch.randn(B, 1, 64, 64, generator=g); t = torch.randint(1, T + 1, (B,), generator=g)
        tr.step(x, c, noise, t, T, ab, lambda: R.draw_shortcut(1, nf))
        t0 = time.perf_counter()
        for _ in range(2):
            tr.step(x, c, noise, t, T, ab, lambda: R.draw_shortcut(1, nf))
        dt = (time.perf_counter() - t0) / 2
        print(f"threads={th}: {dt * 1e3:.0f} ms/step (bs={B}) = {B / dt:.2f} img/s", flush=True)


if __name__ == "__main__":
    main()
