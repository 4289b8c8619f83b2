"""Side-by-side of two tools/conv_micro.py logs (base vs new): built-in tile (t0) or the default
weight-gradient plan, per shape and summed.

    python tools/ab_compare.py <base.log> <new.log> [--wgrad]
"""
import re
import sys


def parse(path, wg):
    d = {}
    pat = r'plan0/s\d+:\s*([\d.]+)us' if wg else r't0:\s*([\d.]+)us'
    for line in open(path):
        if '|' not in line:
            continue
        m = re.search(pat, line)
        if m:
            d[line.split('|')[0].strip()] = float(m.group(1))
    return d


def main():
    wg = "--wgrad" in sys.argv
    a, b = parse(sys.argv[1], wg), parse(sys.argv[2], wg)
    ta = tb = 0.0
    for k in a:
        if k in b:
            print(f"{k:45s} base {a[k]:7.1f} new {b[k]:7.1f}  {a[k] / b[k]:5.2f}x")
            ta += a[k]
            tb += b[k]
    print(f"{'sum':45s} base {ta:7.1f} new {tb:7.1f}  {ta / tb:5.2f}x")


if __name__ == "__main__":
    main()
