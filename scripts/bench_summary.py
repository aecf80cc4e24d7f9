"""One line per bench leg from a bench.py JSON line: value, step, kernel and roofline fractions."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
legs = [('ramsey', d)] + [(k, d[k]) for k in ('config1', 'dds', 'active_reset', 'demod', 'lut', 'rb', 'rb_shaped') if k in d]
for name, a in legs:
    r = a['roofline']
    h = r.get('hbm', r)
    print(name, 'value %.4g' % a['value'], 'step %.4f' % a['ms_per_step'], 'kernel %.4f' % h['kernel_ms'],
          'frac %.3f' % r['frac'], 'hbm_frac %.3f' % h['frac'], 'frac_rocprof', h.get('frac_rocprof'))
