"""Host LLVM IR check: every __hipPushCallConfiguration (the first half of a
triple-chevron kernel launch) reaches its launch -- the kernel's stub, or the
stub's body inlined (hipLaunchKernel) -- within a few basic blocks.  A push
with no launch after it is a launch the compiler dropped (tests/
test_launch_ir.py)."""
import re, sys
LABEL = re.compile(r'^([\w.$-]+):')
def blocks_of(fn_lines):
    blocks = {}; order = []; cur = 'entry'; blocks[cur] = []; order.append(cur)
    for l in fn_lines[1:]:
        m = LABEL.match(l)
        if m:
            cur = m.group(1); blocks[cur] = []; order.append(cur); continue
        if l.strip() and not l.strip().startswith(';'): blocks[cur].append(l.strip())
    return blocks
STUB = re.compile(r'(call|invoke) (void|i32) (@\S*__device_stub__|%)|@hipLaunchKernel\(')
def check(path):
    text = open(path).read().split('\n')
    fns = []; cur = None
    for l in text:
        if l.startswith('define '): cur = [l]; continue
        if cur is not None:
            if l == '}': fns.append(cur); cur = None
            else: cur.append(l)
    pushes = 0; bad = []
    for fn in fns:
        bl = blocks_of(fn)
        for name, ins in bl.items():
            for k, s in enumerate(ins):
                if '@__hipPushCallConfiguration' not in s: continue
                pushes += 1
                rest = ins[k + 1:]
                if any(STUB.search(x) for x in rest): continue
                # the launch (the stub, or the stub's body inlined) must be
                # reachable from the push within a few blocks
                seen = set(); front = [name]; ok = False; first = True
                for depth in range(40):
                    nxt = []
                    for b in front:
                        ins_b = rest if first else bl.get(b, [])
                        if any(STUB.search(x) for x in ins_b): ok = True
                        # (the block's successors: its terminator, which for a
                        # switch spans several lines; only terminators name labels)
                        term = ' '.join(ins_b)
                        for t in re.findall(r'label %([\w.$-]+)', term):
                            if t not in seen: seen.add(t); nxt.append(t)
                    first = False
                    if ok: break
                    front = nxt
                if not ok: bad.append((fn[0][:90], name))
    return pushes, bad
if __name__ == '__main__':
  for p in sys.argv[1:]:
    n, bad = check(p)
    print(p, n, len(bad), bad[:3])
