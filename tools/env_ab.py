"""A/B of the C2 bench step over values of one environment variable (no rebuild):
    python tools/env_ab.py NAME v1 v2 ... [--rounds R]
Each value runs bench.py (20 steps, no CPU baseline) in its own process, alternating over
the values R times; prints the step and per-kernel HIP-event times per run."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1:]
    rounds = 2
    if "--rounds" in args:
        i = args.index("--rounds")
        rounds = int(args[i + 1])
        del args[i:i + 2]
    name, values = args[0], args[1:]
    for _ in range(rounds):
        for v in values:
            env = dict(os.environ)
            if v == "unset":
                env.pop(name, None)
            else:
                env[name] = v
            r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "3",
                                "--cpu-seconds", "0"], env=env, capture_output=True, text=True, timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not line:
                print(f"{name}={v} FAILED rc={r.returncode}", r.stderr[-1500:], flush=True)
                sys.exit(1)
            d = json.loads(line[-1])
            ks = d["kernels_ms"]
            print(f"{name}={v:6s} step {d['ms_per_step']:.4f} ms  " +
                  "  ".join(f"{k.replace('k_', '')} {t * 1e3:.1f}" for k, t in ks.items()), flush=True)


if __name__ == "__main__":
    main()
