"""Summarise a directory of rejected-variant measurements (round-5 `*_rejected/` layouts) as a
markdown table: eval A/B lines (`ab_libs.py`: config, library, median / min ms, bitwise check),
solve-latency runs (`lat_*.json`: ms per single solve, B = 64), 8 192-solve benches (`s5ex_*` / `s5lm_*`:
solves/s) and solve digests (`digest_*`: A and B equal or not).
    python scripts/summarize_rejected.py DIR"""
import glob
import json
import os
import sys


def rows_eval(path):
    out = []
    for line in open(path):
        try:
            d = json.loads(line)
        except ValueError:
            continue
        if "median_ms" in d:
            out.append(f"| {os.path.basename(path)} | {d.get('config')} {d.get('batch', '')} | {d.get('lib', d.get('variant'))} "
                       f"{d.get('tuning', '')} | {d['median_ms']:.4f} | {d.get('min_ms', float('nan')):.4f} |")
        elif "equal" in d:
            out.append(f"| {os.path.basename(path)} | bitwise | {d.get('lib')} vs {d.get('bitwise_equal_to')} | "
                       f"{'equal' if d['equal'] else 'DIFFERENT'} | |")
    return out


def summarize(root):
    lines = [f"## {os.path.relpath(root)}", "", "| file | what | library / variant | median ms (or result) | min ms |",
             "|---|---|---|---|---|"]
    for path in sorted(glob.glob(os.path.join(root, "**", "*"), recursive=True)):
        if os.path.isdir(path) or path.endswith(".md"):
            continue
        rel = os.path.relpath(path, root)
        base = os.path.basename(path)
        try:
            if base.startswith("lat_"):
                d = json.load(open(path))
                b1 = d.get("limited-memory_B1", {}).get("ms_per_solve_call")
                b64 = d.get("limited-memory_B64", {}).get("ms_per_solve_call")
                e1 = d.get("exact_B1", {}).get("ms_per_solve_call")
                lines.append(f"| {rel} | single solve (L-BFGS B=1 / B=64 / exact B=1) | | "
                             f"{b1 and round(b1, 3)} / {b64 and round(b64, 3)} / {e1 and round(e1, 3)} ms | |")
            elif base.startswith("s5"):
                d = json.loads(open(path).read().strip().splitlines()[-1])
                lines.append(f"| {rel} | 8 192 solves ({'exact' if 's5ex' in base else 'L-BFGS'}) | | "
                             f"{d['value'] / 1e3:.1f}k solves/s | |")
            elif base.startswith("digest_"):
                ds = [json.loads(q) for q in open(path) if q.strip()]
                lines.append(f"| {rel} | solve digest | | " + "; ".join(f"{q['hessian']} {q['digest']}" for q in ds) + " | |")
            elif base.endswith(".jsonl"):
                lines += [r.replace(f"| {base} |", f"| {rel} |", 1) for r in rows_eval(path)]
        except (ValueError, KeyError, IndexError) as e:
            lines.append(f"| {rel} | (unparsed: {e}) | | | |")
    return "\n".join(lines) + "\n"


if __name__ == "__main__":
    print(summarize(sys.argv[1]))
