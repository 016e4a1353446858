"""Summarise a rocprofv3 VALU-counter pass (scripts/pmc_valu.sh) for one kernel.

Per dispatch (averaged over the kernel's dispatches): VALU instructions (wave-level, SQ_INSTS_VALU),
the fp64 split (FMA / MUL / ADD / TRANS), VALU busy = SQ_ACTIVE_INST_VALU x 4 cycles over
(#CU x 4 SIMDs x GRBM_GUI_ACTIVE / #XCD) -- the fraction of SIMD cycles with a VALU instruction
in progress -- and, given the pairs per dispatch, instructions per pair.  GRBM_GUI_ACTIVE is the sum
over the 8 XCDs (MI355X_MICROARCH.md, DVFS), so the effective clock is GRBM_GUI_ACTIVE / 8 / duration.
  python tools/summarize_valu.py <csv> <kernel-substring> [--pairs P] [--largest] [--cus 256] [--xcds 8]
"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('kernel')
    ap.add_argument('--pairs', type=float, default=None, help='pairs evaluated per dispatch')
    ap.add_argument('--cus', type=int, default=256)
    ap.add_argument('--xcds', type=int, default=8)
    ap.add_argument('--largest', action='store_true', help='only the dispatch with the most VALU instructions')
    args = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    names = set()
    for r in csv.DictReader(open(args.csv)):
        if args.kernel not in r['Kernel_Name']:
            continue
        names.add(r['Kernel_Name'])
        per[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
        dur[r['Dispatch_Id']] = float(r['End_Timestamp']) - float(r['Start_Timestamp'])
    assert per, f'no dispatch of a kernel matching {args.kernel!r}'
    if args.largest:
        k = max(per, key=lambda d: per[d]['SQ_INSTS_VALU'])
        per = {k: per[k]}
    n = len(per)
    avg = {c: sum(d[c] for d in per.values()) / n for c in next(iter(per.values()))}
    dur_ns = sum(dur[k] for k in per) / n
    gui = avg['GRBM_GUI_ACTIVE'] / args.xcds          # cycles of one XCD over the dispatch
    busy = avg['SQ_ACTIVE_INST_VALU'] * 4 / (args.cus * 4 * gui)
    out = {'kernel': sorted(names), 'dispatches': n,
           'valu_instr_per_dispatch': avg['SQ_INSTS_VALU'],
           'fp64': {k: avg[f'SQ_INSTS_VALU_{k}_F64'] for k in ('FMA', 'MUL', 'ADD', 'TRANS')},
           'gui_cycles_per_xcd': gui, 'valu_busy': round(busy, 4),
           'wave_cycles': avg['SQ_WAVE_CYCLES'], 'busy_cycles': avg['SQ_BUSY_CYCLES'],
           'duration_us': round(dur_ns / 1e3, 1), 'effective_clock_GHz': round(gui / dur_ns, 3)}
    if args.pairs:
        out['valu_instr_per_pair'] = round(avg['SQ_INSTS_VALU'] * 64 / args.pairs, 2)
        out['fp64_instr_per_pair'] = round(sum(out['fp64'].values()) * 64 / args.pairs, 2)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
