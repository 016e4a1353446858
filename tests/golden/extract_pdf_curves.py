"""Extract the golden curves of ``report/figures/gaussian-mixture-comparison.pdf`` (reference).

The figure is produced by ``Gaussian_mixture.ipynb`` cell 85 (json lines ~1139-1158):
left panel = energy distance vs sample2 for m = 1..1000, right panel = cumulative KSD
(``calculate_ksd``, ``code/src/utils/ksd.py:19-27``) of the Stein / gradient-free index
sequences.  Matplotlib writes the polylines as vector paths with 6-decimal point coordinates
(path simplification drops some vertices), so each surviving vertex pins one value
to ~2e-8 relative.

Run in the build container only (reads /root/reference); the output JSON is the committed
fixture ``gm_comparison_curves.json``.  Usage: ``python tests/golden/extract_pdf_curves.py``.
"""
import json
import pathlib
import re
import zlib

PDF = pathlib.Path('/root/reference/report/figures/gaussian-mixture-comparison.pdf')
OUT = pathlib.Path(__file__).with_name('gm_comparison_curves.json')

# Axis calibration read from the same content stream (tick marks):
#   x: tick "0" at x0, tick "200" at x0 + 200*dx  (both panels share dx)
#   y: log10 ticks 10^-1 / 10^0
PANELS = {
    'ed':  {'x0': 65.904961, 'x200': 122.093492, 'y_m1': 113.157456, 'y_0': 248.107605},
    'ksd': {'x0': 426.504721, 'x200': 426.504721 + (122.093492 - 65.904961),
            'y_m1': 113.359527, 'y_0': 250.712197},
}
# stroke colours (matplotlib tab10) -> series, in plot order of cell 85
SERIES = ['naive', 'stein', 'gf_simple_gaussian', 'gf_kde']


def main():
    data = PDF.read_bytes()
    m = re.search(rb'9 0 obj\s*<<[^>]*>>\s*stream\r?\n', data)
    txt = zlib.decompressobj().decompress(data[m.end():]).decode('latin1')
    paths, cur = [], None
    for ln in txt.split('\n'):
        mm = re.match(r'^([-\d.]+) ([-\d.]+) (m|l)$', ln.strip())
        if not mm:
            continue
        x, y = float(mm.group(1)), float(mm.group(2))
        if mm.group(3) == 'm':
            cur = [(x, y)]
            paths.append(cur)
        else:
            cur.append((x, y))
    long_paths = [p for p in paths if len(p) > 100]
    assert len(long_paths) == 8, len(long_paths)
    out = {'source': 'report/figures/gaussian-mixture-comparison.pdf',
           'generated_by': 'Gaussian_mixture.ipynb cell 85', 'curves': {}}
    for panel_i, panel in enumerate(['ed', 'ksd']):
        cal = PANELS[panel]
        dx = (cal['x200'] - cal['x0']) / 200.0
        dy = cal['y_0'] - cal['y_m1']
        for s_i, name in enumerate(SERIES):
            pts = long_paths[panel_i * 4 + s_i]
            series = []
            for x, y in pts:
                k = (x - cal['x0']) / dx
                ik = int(round(k))
                assert abs(k - ik) < 1e-3, (panel, name, x, k)
                log10v = -1.0 + (y - cal['y_m1']) / dy
                series.append([ik + 1, 10.0 ** log10v])   # m = list index + 1
            out['curves'][f'{panel}/{name}'] = series
    OUT.write_text(json.dumps(out, indent=0))
    print('wrote', OUT, {k: len(v) for k, v in out['curves'].items()})


if __name__ == '__main__':
    main()
