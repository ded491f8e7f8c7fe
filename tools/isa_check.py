"""Do the logit-capture (DBG) kernel instances compute exactly what the production instances
compute? (the teacher-forced logit gate runs the DBG instances.)

Every persistent kernel is a template with a trailing `bool DBG`; the DBG instance adds one
predicated store of a logit the production code already computes (persist_common.h
p_dbg_logit). Instruction scheduling and register allocation cannot change an fp32 result; what
could is the backend choosing a different floating-point operation sequence for the same source
-- in practice fmul + fadd pairs contracted into an fma in one instance and not in the other (HIP
compiles with -ffp-contract=fast outside the `contract(off)` epilogues; no reassociation is
enabled). Any such difference changes the instance's COUNT of fp32 operations by opcode. This
tool disassembles the library's gfx950 code objects (the .hip_fatbin section of the built .so,
split into its clang offload bundles) and compares, for every (production, DBG) pair, the
multiset of floating-point value-producing instructions (v_*_f32 / _f64 / _f16, MFMA,
transcendentals, conversions). Integer address arithmetic and moves may differ (the extra store
needs an address); fp operations may not.

usage: python tools/isa_check.py [library.so]   (exit 1 on a mismatch)
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB = os.path.join(REPO, 'real-time-voice-cloning_amd', 'wavernn_amd', 'libwavernn_mi355x.so')
LLVM = '/opt/rocm/lib/llvm/bin'
TARGET = 'hipv4-amdgcn-amd-amdhsa--gfx950'
MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'
# floating-point value-producing opcodes (names carry the type suffix on gfx9)
FP = re.compile(r'^v_(?!cmp|cmpx|cndmask|mov|readlane|readfirstlane|writelane)'
                r'[a-z0-9_]*(f32|f64|f16|bf16|xf32)(_e32|_e64|_dpp|_sdwa)?$|^v_mfma')


def tools_available():
    return all(os.path.exists(os.path.join(LLVM, t))
               for t in ('llvm-objcopy', 'clang-offload-bundler', 'llvm-objdump'))


def kernels_of(lib):
    """{mangled kernel name: [opcode, ...]} over every gfx950 code object in the library."""
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        fb = os.path.join(tmp, 'fatbin')
        subprocess.run([os.path.join(LLVM, 'llvm-objcopy'), f'--dump-section=.hip_fatbin={fb}', lib,
                        os.path.join(tmp, 'lib.copy')], check=True)
        data = open(fb, 'rb').read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        for i in range(len(starts) - 1):
            part = os.path.join(tmp, f'b{i}')
            with open(part, 'wb') as f:
                f.write(data[starts[i]:starts[i + 1]])
            co = part + '.co'
            r = subprocess.run([os.path.join(LLVM, 'clang-offload-bundler'), '--unbundle', '--type=o',
                                f'--input={part}', f'--targets={TARGET}', f'--output={co}'],
                               capture_output=True)
            if r.returncode or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            dis = subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', co], check=True,
                                 capture_output=True, text=True).stdout
            cur = None
            for line in dis.split('\n'):
                m = re.match(r'^[0-9a-f]+ <(\S+)>:', line)
                if m:
                    cur = m.group(1)
                    out[cur] = []
                    continue
                s = line.strip()
                if cur and s[:2] in ('v_', 's_', 'ds', 'bu', 'gl', 'fl', 'sc'):
                    out[cur].append(s.split()[0])
    return out


def dbg_pairs(kern):
    """(production name, DBG name) pairs: the DBG flag is the last template argument, except in
    k_persist, whose last one is SP (the sparse instances, round 6): DBG is the one before it."""
    pairs = []
    for name in kern:
        if '9k_persistI' in name:
            m = re.match(r'^(.*)Lb1E(Lb[01]EEEvN.*)$', name)
        else:
            m = re.match(r'^(.*)Lb1E(EEvN.*)$', name)
        if m and (m.group(1) + 'Lb0E' + m.group(2)) in kern:
            pairs.append((m.group(1) + 'Lb0E' + m.group(2), name))
    return pairs


def fp_hist(ops):
    return collections.Counter(o for o in ops if FP.match(o))


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else LIB
    kern = kernels_of(lib)
    pairs = dbg_pairs(kern)
    bad = 0
    for prod, dbg in sorted(pairs):
        a, b = fp_hist(kern[prod]), fp_hist(kern[dbg])
        diff = {k: (a[k], b[k]) for k in set(a) | set(b) if a[k] != b[k]}
        short = re.sub(r'_ZN4wrnn\d+', '', prod)[:60]
        print(f'{short:62s} fp ops {sum(a.values()):5d} / {sum(b.values()):5d}  '
              f'{"same" if not diff else "DIFFERENT " + str(diff)}')
        bad += bool(diff)
    print(f'{len(pairs)} production / DBG pairs, {bad} with different fp arithmetic')
    return 1 if bad or not pairs else 0


if __name__ == '__main__':
    sys.exit(main())
