#!/usr/bin/env python3
"""Program order of two sets of LDS accesses in a kernel's line-annotated disassembly (measurement infra, CPU only).

Used for the round-5 fault (r05f): did the compiler schedule collide()'s geom-centre stores above the
arm mass-matrix loop's reads of the same phase-local region (the hand-off the missing SYNC() left unordered)?

usage: llvm-objdump -d -l --no-show-raw-insn CODE_OBJECT > dis.txt
       python tools/lds_order_probe.py dis.txt READ_LINES WRITE_LINES [KERNEL_SUBSTRING]
       (READ_LINES / WRITE_LINES: fm_device.hpp line ranges "a-b"; default kernel: step_kernel<float, FixedDims<2, 8>, false>)
"""
import re, sys
path = sys.argv[1]; ksub = sys.argv[4] if len(sys.argv) > 4 else 'ILi2ELi8ELb0EEELb0EEE'; rd = tuple(map(int, sys.argv[2].split('-'))); wr = tuple(map(int, sys.argv[3].split('-')))
lines = open(path).read().splitlines()
func = None; src = None; out = []
for l in lines:
    m = re.match(r'^[0-9a-f]+ <(.*)>:', l)
    if m: func = m.group(1); continue
    m = re.match(r'^; .*fm_device\.hpp:(\d+)', l)
    if m: src = int(m.group(1)); continue
    if l.startswith('; '): src = None; continue
    m = re.match(r'^\s+(ds_\w+|s_waitcnt|s_cbranch\w*|s_branch)\b(.*?)//\s*([0-9A-F]+):', l)
    if m and func and ksub in func:
        out.append((int(m.group(3), 16), m.group(1), src, m.group(2).strip()))
reads = [x for x in out if x[1].startswith('ds_read') and x[2] is not None and rd[0] <= x[2] <= rd[1]]
writes = [x for x in out if x[1].startswith('ds_write') and x[2] is not None and wr[0] <= x[2] <= wr[1]]
print('mass-matrix reads', len(reads), [hex(x[0]) for x in reads[:3]], '..', [hex(x[0]) for x in reads[-3:]])
print('gx writes', len(writes), [hex(x[0]) for x in writes[:3]], '..', [hex(x[0]) for x in writes[-3:]])
lr = max(x[0] for x in reads); fw = min(x[0] for x in writes)
print('last mass-matrix read', hex(lr), 'first gx write', hex(fw), '-> gx write issued before the last read:', fw < lr)
for x in out:
    if fw - 0x40 <= x[0] <= lr + 0x10 and (x[1].startswith('ds_') or x[1].startswith('s_')):
        print(hex(x[0]), x[1], x[2], x[3][:60])
