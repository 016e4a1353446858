"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reads exactly half the bytes of a
wide coalesced streaming read -> doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Both
counters are in KiB.  Usage:
  python tools/summarize_pmc.py <fetch_csv> <write_csv> <config> [--kernel greedy_step] [--out profiles/pmc_traffic.json]
"""
import argparse
import collections
import csv
import json
import os


def load(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r['Kernel_Name'], r['Counter_Name'])].append(float(r['Counter_Value']))
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch_csv')
    ap.add_argument('write_csv')
    ap.add_argument('config')
    ap.add_argument('--kernel', default='greedy_step_ct')
    ap.add_argument('--exclude', default=', true, ')   # template arg DIAG=true -> diagonal launch
    ap.add_argument('--out', default='profiles/pmc_traffic.json')
    ap.add_argument('--source', default='', help='which pass this was (round, script, commit): kept in the record')
    args = ap.parse_args()
    f, w = load(args.fetch_csv), load(args.write_csv)

    def pick(agg, counter):
        vals = [v for (k, c), v in agg.items() if c == counter and args.kernel in k and args.exclude not in k]
        names = [k for (k, c) in agg if c == counter and args.kernel in k and args.exclude not in k]
        assert len(vals) == 1, names
        return names[0], sum(vals[0]) / len(vals[0]), len(vals[0]), vals[0]
    kname, fetch_kib, nf, fl = pick(f, 'FETCH_SIZE')
    _, write_kib, nw, wl = pick(w, 'WRITE_SIZE')
    rec = {'kernel': kname, 'launches_fetch': nf, 'launches_write': nw,
           # each dispatch separately (MB, corrected): the persistent kernels' reads are mostly the exchange's
           # polls of remote records and vary with how many polls each step takes
           'read_MB_per_dispatch': [round(2 * v / 1024, 1) for v in fl],
           'write_MB_per_dispatch': [round(v / 1024, 1) for v in wl],
           'note': ('8-B-per-lane loads (dwordx2) are outside the guide\'s calibration; the same 128-B-request '
                    'x2 correction is applied') if 'persistent' in kname else '',
           'FETCH_SIZE_KiB_per_launch': fetch_kib, 'WRITE_SIZE_KiB_per_launch': write_kib,
           'read_bytes_per_launch': 2 * fetch_kib * 1024, 'write_bytes_per_launch': write_kib * 1024,
           'hbm_bytes_per_launch': (2 * fetch_kib + write_kib) * 1024,
           'correction': 'FETCH_SIZE x2 (gfx950 half-count of wide coalesced reads); KiB -> bytes'}
    if args.source:
        rec['source'] = args.source
    out = json.load(open(args.out)) if os.path.exists(args.out) else {}
    out[args.config] = rec
    json.dump(out, open(args.out, 'w'), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == '__main__':
    main()
