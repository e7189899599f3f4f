"""A/B of library builds / host-build switches on one GPU box: bench.py runs per variant,
interleaved over rounds, one summary line per run (value, ms/frame, one-launch kernel ms).

usage: tools/ab_bench.py PREFIX CONFIG STEPS ROUNDS NAME[:ENV=VAL[,ENV=VAL...]] ...
  (a key opt.NAME passes --option NAME=VAL to bench.py instead of setting the environment)
  e.g. tools/ab_bench.py r05b c3 1000 2 base:MYRT_LIB=build_variants/libmyrt_base.so main
Each run: python bench.py --config CONFIG --steps STEPS --no-cpu-baseline --no-side-paths, its
JSON line written to gpurun_out/PREFIX_bench_CONFIG_NAME[_k].json and summarised on stdout.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    prefix, cfg, steps, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    variants = []
    for spec in sys.argv[5:]:
        name, _, envs = spec.partition(":")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        variants.append((name, env))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    rows = []
    for r in range(rounds):
        for name, env in variants:
            e = dict(os.environ)
            opts = []
            for k, v in env.items():
                if k.startswith("opt."):                 # opt.NAME=VALUE: bench --option NAME=VALUE
                    opts += ["--option", f"{k[4:]}={v}"]
                else:
                    e[k] = os.path.join(ROOT, v) if k == "MYRT_LIB" else v
            cmd = [sys.executable, "bench.py", "--config", cfg, "--steps", str(steps), "--no-cpu-baseline",
                   "--no-side-paths"] + opts
            p = subprocess.run(["timeout", "-k", "10", "300"] + cmd, cwd=ROOT, env=e, capture_output=True, text=True)
            if p.returncode != 0:
                print(f"{name}: rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(p.returncode)
            line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
            out = os.path.join(ROOT, "gpurun_out", f"{prefix}_bench_{cfg}_{name}{'_' + str(r) if r else ''}.json")
            with open(out, "w") as f:
                f.write(line + "\n")
            j = json.loads(line)
            km = (j.get("roofline") or {}).get("kernel_ms")
            row = f"{os.path.basename(out):42s} {j['value']:9.1f} Mrays/s  {j['ms_per_step']:.4f} ms/frame  kernel {km} ms"
            print(row, flush=True)
            rows.append(row)
    with open(os.path.join(ROOT, "gpurun_out", f"{prefix}_ab_{cfg}.txt"), "w") as f:
        f.write(f"{prefix} A/B {cfg}, {steps} frames, variants: " +
                "; ".join(f"{n}={v}" for n, v in variants) + "\n" + "\n".join(rows) + "\n")


if __name__ == "__main__":
    main()
