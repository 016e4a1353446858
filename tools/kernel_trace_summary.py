"""Median duration of one kernel's TIMED dispatches from a rocprofv3 --kernel-trace CSV.

bench.py enqueues, per kernel of interest, `warmup` untimed dispatches, then `steps` timed ones
(then, for the thin workload, the end-to-end drop-in calls).  This picks dispatches
[warmup, warmup + steps) of the kernels whose name contains `--kernel` (in dispatch order) and
prints their median / mean / min / max, so the bench line's `kernel_median_us` can be checked
against the profiler's own clock:

  python tools/kernel_trace_summary.py gpurun_out/prof/run_kernel_trace.csv --kernel greedy_persistent \
      --warmup 2 --steps 10 [--json out.json]
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace_csv')
    ap.add_argument('--kernel', required=True)
    ap.add_argument('--warmup', type=int, default=0)
    ap.add_argument('--steps', type=int, default=None)
    ap.add_argument('--exclude', default=None, help='skip kernel names containing this')
    ap.add_argument('--json', default=None)
    args = ap.parse_args()
    rows = []
    with open(args.trace_csv) as f:
        for r in csv.DictReader(f):
            name = r['Kernel_Name']
            if args.kernel not in name or (args.exclude and args.exclude in name):
                continue
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']) - int(r['Start_Timestamp']), name))
    rows.sort()
    sel = rows[args.warmup:] if args.steps is None else rows[args.warmup:args.warmup + args.steps]
    if not sel:
        raise SystemExit(f'no dispatches of {args.kernel!r} in [{args.warmup}, +{args.steps})')
    us = [d / 1e3 for _, d, _ in sel]
    out = {'kernel': sel[0][2], 'dispatches_total': len(rows), 'selected': [args.warmup, args.warmup + len(sel)],
           'median_us': statistics.median(us), 'mean_us': statistics.fmean(us), 'min_us': min(us), 'max_us': max(us),
           'all_us_in_order': [round(d / 1e3, 1) for _, d, _ in rows]}
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
