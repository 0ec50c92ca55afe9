"""CPU ORACLE -- test infrastructure only.

This package is a NumPy restatement of the reference's hot path
(Dostenlinus/Aiyagari-HARK, ``Aiyagari_Support.py``) plus the econ-ark (HARK) 0.12
library semantics the reference calls into (HARK is not vendored in the reference
and is not installed here).

It is the *checker*: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product package ``aiyagari_hark_amd`` must
never import anything from here.

Parity status: the reference has no tests, fixtures or golden vectors and HARK 0.12
cannot be imported or installed offline, so this restatement is pinned only by the
closed forms and recorded notebook outputs listed in SURVEY.md §4/§6 ("parity
partially pinned": closed-form steady state, Markov-matrix identities, Table II
statistical anchors).  See DESIGN.md §Oracle.
"""
