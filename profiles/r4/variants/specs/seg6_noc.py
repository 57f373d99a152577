# events before the refill: no copy of the row (4 v_mov a row) at the cost of
# the refill waiting for an event row's work; plus the 128-bit tie
import runpy, os
TIE = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "seg5_tie.py"))["TIE"]
NOC = [("""    const uint64_t evm = __ballot(wpos >= rs && wpos < rs + 1024u);
    uint4 we = w;
    // the folds complete before the refill (else they sink past the event
    // branch's join and the refill needs a fresh register: see pin below)
    asm volatile("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(we.x), "+v"(we.y), "+v"(we.z), "+v"(we.w));
    __builtin_amdgcn_sched_barrier(0);
    q = buf_load16(rn, no);
    __builtin_amdgcn_sched_barrier(0);
    if (evm) events(we, rs, wpos, evm);
""", """    const uint64_t evm = __ballot(wpos >= rs && wpos < rs + 1024u);
    asm volatile("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3));
    if (evm) events(w, rs, wpos, evm);
    __builtin_amdgcn_sched_barrier(0);
    q = buf_load16(rn, no);
    __builtin_amdgcn_sched_barrier(0);
""")]
SUBS = TIE + NOC
