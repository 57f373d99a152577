# timing only (wrong words): k_seg_stream without its event work (no H placements at event rows),
# to bound what the events cost the record stream
SUBS = [
    ("    if (evh) events(w, rs, wpos, evh);\n", "    (void)evh;\n"),
]
