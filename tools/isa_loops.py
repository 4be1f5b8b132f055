"""Per-loop instruction mix of one kernel in a disassembly (llvm-objdump -d
--no-show-raw-insn): every backward branch closes a loop; for each loop the
static counts of MFMA / VALU / SALU / LDS / VMEM / waitcnt / branch
instructions between its target and the branch.
  python tools/isa_loops.py /tmp/conv.s 'conv_patch_kernelILi2ELi2ELi3ELi1ELb1ELb0ELi4E'"""
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
text = open(src).read()
funcs = re.split(r'\n(?=[0-9a-f]+ <)', text)
for f in funcs:
    m = re.match(r'([0-9a-f]+) <(.*?)>:', f)
    if not m or pat not in m.group(2):
        continue
    print(m.group(2))
    ins = []
    for l in f.split('\n')[1:]:
        mm = re.match(r'\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):(.*)', l)
        if mm:
            ins.append((int(mm.group(3), 16), mm.group(1), mm.group(2) + mm.group(4)))
    addr = {a: i for i, (a, _, _) in enumerate(ins)}

    def cat(op):
        if op.startswith('v_mfma'):
            return 'mfma'
        if op.startswith('v_'):
            return 'valu'
        if op.startswith('s_waitcnt'):
            return 'wait'
        if op.startswith('s_cbranch') or op.startswith('s_branch'):
            return 'br'
        if op.startswith('s_'):
            return 'salu'
        if op.startswith('ds_'):
            return 'lds'
        if op.startswith(('buffer_', 'global_', 'flat_', 'scratch_')):
            return 'vmem'
        return 'other'
    for i, (a, op, args) in enumerate(ins):
        if op.startswith('s_cbranch') or op == 's_branch':
            t = re.search(r'<.*\+0x([0-9a-f]+)>', args)
            if not t:
                continue
            tgt = int(m.group(1), 16) + int(t.group(1), 16)
            j = addr.get(tgt)
            if j is None or j > i:
                continue
            cnt = {}
            for _, o, _ in ins[j:i + 1]:
                c = cat(o)
                cnt[c] = cnt.get(c, 0) + 1
            if cnt.get('mfma', 0) == 0 and '-a' not in sys.argv:
                continue
            print(f'  loop [{j}..{i}] {i - j + 1} instrs: ' +
                  ' '.join(f'{k}={v}' for k, v in sorted(cnt.items())))
    break
