import runpy, os
LDSCOL = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "seg2_ldscol.py"))["LDSCOL"]
DEEP = [
("""  __amdgpu_buffer_rsrc_t rc = unit_rsrc(u);
  uint4 q0 = buf_load16(rc, lane * 16u), q1 = buf_load16(rc, 1024u + lane * 16u),
        q2 = buf_load16(rc, 2048u + lane * 16u), q3 = buf_load16(rc, 3072u + lane * 16u);
""", """  __amdgpu_buffer_rsrc_t rc = unit_rsrc(u);
  uint4 q0 = buf_load16(rc, lane * 16u), q1 = buf_load16(rc, 1024u + lane * 16u),
        q2 = buf_load16(rc, 2048u + lane * 16u), q3 = buf_load16(rc, 3072u + lane * 16u);
  uint4 p0 = buf_load16(rc, 4096u + lane * 16u), p1 = buf_load16(rc, 5120u + lane * 16u),
        p2 = buf_load16(rc, 6144u + lane * 16u), p3 = buf_load16(rc, 7168u + lane * 16u);
"""),
("""  for (;;) {
    const uint64_t gs = geo.a0 + (u << kU) + ((uint64_t)g << 12);
    const uint64_t wpos = win_pos(wraw, wfirst);
    const bool lastg = g == (1u << (kU - 12)) - 1u;  // the unit's last 4 KiB group
    // the next group: this unit's, or unit un's first; its events' window
    const uint32_t gcnt = (uint32_t)__popcll(__ballot(wpos < gs + 4096u));  // the group's events
    const uint64_t nf = lastg ? (uint64_t)first_ev[un < M ? un : M] : wfirst + gcnt;
    const __amdgpu_buffer_rsrc_t rn = lastg ? unit_rsrc(un) : rc;
    const uint32_t no = lastg ? lane * 16u : ((g + 1) << 12) + lane * 16u;
    // each refill pinned right after its row's fold (as k_crc_grp's kPin):
    // hipcc otherwise hoists it into a fresh register and copies that at the
    // loop latch, which waits for the load (vmcnt(0))
    wraw = win_issue(nf);
    row(q0, gs, wpos, rn, no);
    row(q1, gs + 1024u, wpos, rn, no + 1024u);
    row(q2, gs + 2048u, wpos, rn, no + 2048u);
    row(q3, gs + 3072u, wpos, rn, no + 3072u);
    // the group's event words and the previous unit's raw CRC (if one is
    // pending): two buffer stores every group, straight-line code (a store
    // behind a branch makes hipcc's vmcnt waits count the path without it)
    buf_store_u32(buf_range(ev_h + wfirst, gcnt * 4u), hv, lane * 4u);
    buf_store_u32(buf_range(unit_raw + u_pend, ur_bytes), ur_pend, lane * 4u);
    ur_bytes = 0;
    wfirst = nf;
    if (lastg) {
      ur_pend = wave_xor(place(c0, c1, c2, c3));
""", """  // two groups in flight: group gg's rows in r*, refilled with group gg + 2
  auto group = [&](uint4 &r0, uint4 &r1, uint4 &r2, uint4 &r3, uint32_t gg, __amdgpu_buffer_rsrc_t rr, uint32_t ro) {
    const uint64_t gs = geo.a0 + (u << kU) + ((uint64_t)gg << 12);
    const uint64_t wpos = win_pos(wraw, wfirst);
    const bool lastg = gg == (1u << (kU - 12)) - 1u;
    const uint32_t gcnt = (uint32_t)__popcll(__ballot(wpos < gs + 4096u));
    const uint64_t nf = lastg ? (uint64_t)first_ev[un < M ? un : M] : wfirst + gcnt;
    wraw = win_issue(nf);
    const uint32_t no = ro + lane * 16u;
    row(r0, gs, wpos, rr, no);
    row(r1, gs + 1024u, wpos, rr, no + 1024u);
    row(r2, gs + 2048u, wpos, rr, no + 2048u);
    row(r3, gs + 3072u, wpos, rr, no + 3072u);
    buf_store_u32(buf_range(ev_h + wfirst, gcnt * 4u), hv, lane * 4u);
    buf_store_u32(buf_range(unit_raw + u_pend, ur_bytes), ur_pend, lane * 4u);
    ur_bytes = 0;
    wfirst = nf;
  };
  for (;;) {
    const bool second = g != 0;  // groups 2, 3: refills from the next unit
    const __amdgpu_buffer_rsrc_t rn = second ? unit_rsrc(un) : rc;
    const uint32_t ro = second ? 0u : 2u << 12;
    group(q0, q1, q2, q3, g, rn, ro);
    group(p0, p1, p2, p3, g + 1, rn, ro + 4096u);
    const bool lastg = second;
    if (lastg) {
      ur_pend = wave_xor(place(c0, c1, c2, c3));
"""),
("""      un = unit_of(uni(kv));
      if (lane == 0) kv = atomicAdd(&s_next, 1u);
    } else {
      g++;
    }
  }
}
""", """      un = unit_of(uni(kv));
      if (lane == 0) kv = atomicAdd(&s_next, 1u);
    } else {
      g = 2;
    }
  }
}
"""),
]
SUBS = LDSCOL + DEEP
