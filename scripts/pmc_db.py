#!/usr/bin/env python3
"""Per-kernel PMC averages from a rocprofv3 results database (.db): python scripts/pmc_db.py <db> [substr]"""
import collections
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    q = '''select k.kernel_name, i.name, p.event_id, p.value from rocpd_pmc_event p
           join rocpd_info_pmc i on p.pmc_id = i.id
           join rocpd_kernel_dispatch d on d.event_id = p.event_id
           join rocpd_info_kernel_symbol k on k.id = d.kernel_id'''
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for kname, name, ev, val in c.execute(q):
        if sub and sub not in kname:
            continue
        per[kname][name] += val
        disp[kname].add(ev)
    for k, d in per.items():
        n = len(disp[k])
        print(k[:60], f"dispatches={n}", {m: round(v / n) for m, v in sorted(d.items())})


if __name__ == "__main__":
    main()
