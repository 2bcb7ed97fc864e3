"""CPU oracle for the MultiAgentGraphConstrainEnv step path — TEST INFRASTRUCTURE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from here, and only as the checker / the timed CPU
baseline. The product (``gs-marl_amd/``) never imports, links or executes it.

Parity status: UNPINNED with respect to the true GS-MARL numerics — the
reference's hot-path source is absent (``/root/reference/readme.md:1``) and it
ships no tests or fixtures. Pinned pieces: Philox4x32-10 vs the Random123 KATs;
analytic physics KATs; two independent restatements (``mpe_ref`` object-per-
entity, ``batch_ref`` vectorised) that must agree. See DESIGN.md §3.
"""
