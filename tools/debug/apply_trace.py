"""Debug only: patch temporary per-iteration s_memrealtime stamps into
k_pcompress (pcompress.h) plus a dietgpu_debug_set() hook (codec.hip), for
tools/debug/trace.py.  Never committed into the product build: apply, build,
run the trace on the GPU box, then git checkout the two sources."""
p='/root/repo/dietgpu_fork_amd/csrc/pcompress.h'
s=open(p).read()
def sub(old,new,cnt=1):
    global s
    assert s.count(old)==cnt, (old[:70], s.count(old))
    s=s.replace(old,new)
sub('''  int pb;
  bool useChecksum;
};

// One item''','''  int pb;
  bool useChecksum;
  uint64_t* dbg;
};

// One item''')
sub('''  // this workgroup's item of round r''','''  uint32_t itn = 0;
  auto stamp = [&](uint32_t k) { if (tid == 0 && A().dbg && itn < 8) A().dbg[(blockIdx.x * 8 + itn) * 8 + k] = __builtin_amdgcn_s_memrealtime(); };
  // this workgroup's item of round r''')
sub('''  while (true) {
    const bool hasE''','''  while (true) {
    stamp(0);
    const bool hasE''')
sub('''      if (hasE) encodeDone(E);
    }''','''      if (hasE) encodeDone(E);
    }
    stamp(1);''')
sub('''    if (hasE) place(itemOf(iE, A(), IN()), poisonE, ckE);''','''    stamp(2);
    if (hasE) place(itemOf(iE, A(), IN()), poisonE, ckE);
    stamp(3);''')
sub('''      iN = itemAt(++round);
    }''','''      iN = itemAt(++round);
    }
    stamp(4);
    ++itn;''')
sub('''      if (lane == 0) stateS = ok ? 0u : 1u;
    }''','''      if (lane == 0) stateS = ok ? 0u : 1u;
    }
    stamp(6);''')
sub('''      if (lane < nk) preE[lane] = excl + inc - r;''','''      if (lane < nk) preE[lane] = excl + inc - r;
      stamp(7);''')
open(p,'w').write(s)
p='/root/repo/dietgpu_fork_amd/csrc/codec.hip'
s=open(p).read()
s=s.replace('''  a.useChecksum = useChecksum;
  prof::Scope p("compress", s);''','''  a.useChecksum = useChecksum;
  a.dbg = gDbg;
  prof::Scope p("compress", s);''')
s=s.replace('''// Single-pass compression (k_pcompress''','''uint64_t* gDbg = nullptr;
// Single-pass compression (k_pcompress''')
s=s.rstrip()+'''
extern "C" void dietgpu_debug_set(void* p) { dietgpu::gDbg = (uint64_t*)p; }
'''
open(p,'w').write(s)
