"""R-hat table of every reference-protocol MH run recorded this round.

Reads the SBC records (scripts/mcmc_calibration.py) and the training re-score (scripts/train_protocol.py)
and writes one markdown table: per run, the TAC count, how many runs the reference's own check
(mcmc.py:183-194, R-hat > 1.02 on any variable) flags, the median and max of rhat_max, and min ESS where
recorded.  Usage: python scripts/rhat_table.py [out.md]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
RUNS = [
    ('SBC, PyMC element ratio (sweep start), 4 x (20k + 40k tune)', 'profiles/r03/mcmc/sbc_pymc_20k40k.json'),
    ('SBC, PyMC element ratio, 4 x (40k + 80k tune)', 'profiles/r03/mcmc/sbc_pymc_40k80k.json'),
    ('SBC, textbook element ratio (running state), 4 x (20k + 40k tune)', 'profiles/r03/mcmc/sbc_textbook_20k40k.json'),
]


def main(out):
    rows = []
    for name, path in RUNS:
        d = json.load(open(os.path.join(ROOT, path)))
        per = d['per_tac']
        rh = np.array([p['rhat_max'] for p in per])
        ess = [p.get('ess_min') for p in per if p.get('ess_min') is not None]
        rows.append((name, path, len(per), int((rh > 1.02).sum()), float(np.median(rh)), float(rh.max()),
                     float(min(ess)) if ess else None))
    tr = json.load(open(os.path.join(ROOT, 'profiles/r03/train/summary.json')))
    for key, name in (('mcmc_rhat_max', 'iDDPM re-score TACs, PyMC element ratio, 4 x (20k + 40k tune)'),
                      ('mcmc_textbook_rhat_max', 'iDDPM re-score TACs, textbook element ratio, 4 x (20k + 40k tune)')):
        rh = np.array([e[key] for e in tr['eval']])
        rows.append((name, 'profiles/r03/train/summary.json', len(rh), int((rh > 1.02).sum()), float(np.median(rh)),
                     float(rh.max()), None))
    lines = ['| run | TACs | flagged (R-hat > 1.02) | median rhat_max | max rhat_max | min ESS | record |',
             '|---|---|---|---|---|---|---|']
    for name, path, n, fl, med, mx, ess in rows:
        lines.append(f'| {name} | {n} | {fl} | {med:.4f} | {mx:.4f} | {"" if ess is None else f"{ess:.0f}"} | `{path}` |')
    text = '\n'.join(lines) + '\n'
    with open(out, 'w') as f:
        f.write('# R-hat of the MH baseline runs, round 3\n\nRank-normalised split R-hat (`metrics.rhat`, ArviZ\'s '
                'definition; the reference flags R-hat > 1.02, mcmc.py:183-194). rhat_max is the max over the 96 '
                'variables of one TAC.\n\n' + text)
    print(text)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, 'profiles/r03/mcmc/rhat_table.md'))
