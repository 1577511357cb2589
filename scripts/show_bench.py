#!/usr/bin/env python3
"""One line per bench log: value, ms/step, status histogram, pass times."""
import json
import sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f, round(d['value']), round(d['ms_per_step'], 2), d.get('status_hist'),
                  {k: round(v, 2) for k, v in d.get('pass_ms', {}).items() if v > 0.05},
                  'frac', round(d.get('roofline', {}).get('frac', 0), 4))
