import sys,json
for l in open(sys.argv[1]):
    try: d=json.loads(l)
    except: continue
    if 'query' not in d: print(d); continue
    print(f"{d['query']:5s} {d['set']:40s} p50 {d['p50_ms']:.4f} f {d['filter_ms']:.4f} a {d['agg_ms']:.4f} same {d['same_as_first']}")
