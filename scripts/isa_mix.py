"""Static instruction mix of k_render instantiations in a saved .s (make asm): python scripts/isa_mix.py FILE.s [filter]"""
import collections
import re
import subprocess
import sys

txt = open(sys.argv[1]).read().splitlines()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cur, funcs = None, collections.OrderedDict()
for line in txt:
    m = re.match(r'^(_Z\S+):', line)
    if m:
        cur = m.group(1)
        funcs[cur] = []
        continue
    if cur and line.startswith('\t') and not line.startswith('\t.') and not line.startswith('\t;'):
        funcs[cur].append(line.strip())
    if cur and line.startswith('.Lfunc_end'):
        cur = None
for name, ins in funcs.items():
    dn = subprocess.run(['c++filt', name], capture_output=True, text=True).stdout.strip()
    m = re.search(r'k_render<([^>]*)>', dn)
    if not m:
        continue
    t = m.group(1).replace(' ', '')
    if flt not in t:
        continue
    c = collections.Counter(i.split()[0] for i in ins if i.split())
    grp = lambda p: sum(v for k, v in c.items() if k.startswith(p))
    print(f"{t:55s} n {len(ins):5d} valu {grp('v_'):5d} salu {grp('s_'):5d} fma_mix {c['v_fma_mix_f32']:3d} "
          f"v_fma {c['v_fma_f32']:3d} s_load16 {c['s_load_dwordx16']:2d} waitcnt {c['s_waitcnt']:3d} "
          f"v_mov {grp('v_mov'):4d} s_mov {grp('s_mov'):4d} readlane {grp('v_readfirstlane')+grp('v_readlane')}")
