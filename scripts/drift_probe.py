"""Config 2's in-run drift: per-launch kernel times of the
product hash kernel, back to back vs. with idle gaps, and with the device's
clocks sampled between launches.

    python scripts/drift_probe.py --config cfg2 --launches 40

Prints one JSON line per schedule with every launch's HIP-event time (ms):
  back_to_back   launches queued with no host wait (bench.py's timed loop);
  gap_sync       host synchronize + sleep(gap) before each launch;
  after_flush    before each launch a 512 MiB streaming write to another
                 buffer (leaves dirty lines in L2 / the Infinity Cache, as a
                 previous launch's coordinate stores do);
  coords_rotate  back to back, each launch writing a different coordinate
                 buffer (4 in rotation).
"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def smi_clocks():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True, text=True,
                             timeout=20).stdout
        card = next(iter(json.loads(out).values()))
        return {k: v for k, v in card.items() if "clock" in k.lower() and ("sclk" in k or "mclk" in k or "fclk" in k)}
    except Exception as e:  # noqa: BLE001 — diagnostic only
        return {"error": str(e)[:80]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--objects", type=int, default=10_000_000)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--gap-ms", type=float, default=5.0)
    a = ap.parse_args()
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import synth
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    types, blob, base, lens = synth.make_batch_device(a.config, a.objects, device=dev)
    A = len(types)
    coords = [torch.empty((a.objects, A), dtype=torch.int64, device=dev) for _ in range(4)]
    scratch = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    for _ in range(3):
        hdx.hash_batch(types, blob, base, lens, coords=coords[0], stream=stream)
    torch.cuda.synchronize()

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def run(schedule):
        evs = [(ev(), ev()) for _ in range(a.launches)]
        t0 = time.perf_counter()
        for k, (s, e) in enumerate(evs):
            if schedule == "gap_sync":
                torch.cuda.synchronize()
                time.sleep(a.gap_ms / 1e3)
            elif schedule == "after_flush":
                scratch.fill_(k & 0xff)
            s.record(stream)
            hdx.hash_batch(types, blob, base, lens, coords=coords[k % 4 if schedule == "coords_rotate" else 0],
                           stream=stream)
            e.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ms = [round(s.elapsed_time(e), 4) for s, e in evs]
        return {"schedule": schedule, "config": a.config, "objects": a.objects, "kernel_ms": ms,
                "first5_mean": round(sum(ms[:5]) / 5, 4), "last20_mean": round(sum(ms[-20:]) / 20, 4),
                "wall_ms_per_launch": round(wall / a.launches * 1e3, 4)}

    print(json.dumps({"clocks_before": smi_clocks()}), flush=True)
    for sch in ("back_to_back", "gap_sync", "after_flush", "coords_rotate", "back_to_back"):
        print(json.dumps(run(sch)), flush=True)
    print(json.dumps({"clocks_after": smi_clocks()}), flush=True)


if __name__ == "__main__":
    main()
