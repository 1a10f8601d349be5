import json, sys
for f in sys.argv[1:]:
    try:
        l = [x for x in open(f) if x.startswith('{')][-1]
    except Exception as e:
        print(f, 'no json', e); continue
    d = json.loads(l); r = d['roofline']
    print(f.split('/')[-1], 'value', round(d['value']), 'ms/step', round(d['ms_per_step'], 3), r.get('formats'), 'frac', round(r['frac'], 3))
    for k, v in r['launches'].items(): print('    ', k, v)
    for k in ('hvp_warm_us', 'reorth'):
        if d.get(k) is not None: print('    ', k, d[k])
