"""Instruction mix of a kernel's loops from a hipcc -save-temps assembly file.

    python tools/isa_loops.py <file.s> <kernel-symbol-substring>

For every backward branch (a loop) prints its label range and the count of MFMA, VALU, LDS, VMEM, SALU and
s_waitcnt instructions in the body, plus the MFMA issue cycles (32 for 32x32x16 bf16, 16 for 16x16x32 bf16 and
16x16x4 f32... per the microarch guide's constants) and a rough VALU issue estimate at 4 cycles per instruction for
one wave alone on its SIMD.
"""
import collections
import re
import sys

MFMA_CYC = {'v_mfma_f32_32x32x16_bf16': 32, 'v_mfma_f32_16x16x32_bf16': 16, 'v_mfma_f32_16x16x4_f32': 32,
            'v_mfma_f32_32x32x2_f32': 64}


def kernel_lines(path, sub):
    text = open(path).read().split('\n')
    start = next(i for i, l in enumerate(text) if re.match(r'^_Z\S*%s\S*:' % re.escape(sub), l))
    end = next(i for i in range(start, len(text)) if text[i].startswith('.Lfunc_end'))
    return text[start:end]


def classify(op):
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('buffer_', 'global_', 'flat_')):
        return 'vmem'
    if op.startswith('s_waitcnt'):
        return 'wait'
    if op.startswith('s_barrier'):
        return 'barrier'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('v_'):
        return 'valu'
    return 'other'


def main():
    lines = kernel_lines(sys.argv[1], sys.argv[2])
    labels = {}
    insts = []
    for l in lines:
        t = l.strip()
        m = re.match(r'^(\.LBB\d+_\d+):', t)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        if not t or t.startswith(('.', ';', '//')) or t.endswith(':'):
            continue
        insts.append(t)
    total = collections.Counter(classify(i.split()[0]) for i in insts)
    print('kernel: %d instructions %s' % (len(insts), dict(total)))
    for k, ins in enumerate(insts):
        op = ins.split()[0]
        if op.startswith('s_cbranch') or op == 's_branch':
            tgt = ins.split()[-1]
            if tgt in labels and labels[tgt] <= k:
                body = insts[labels[tgt]:k + 1]
                c = collections.Counter(classify(i.split()[0]) for i in body)
                mcyc = sum(MFMA_CYC.get(i.split()[0], 0) for i in body)
                print('loop %s [%d..%d] %d inst: %s  mfma_cycles %d  valu_issue~%d' % (
                    tgt, labels[tgt], k, len(body), dict(c), mcyc, 4 * c['valu']))


if __name__ == '__main__':
    main()
