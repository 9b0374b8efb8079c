"""CPU oracle for the valuation path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
import this package, and only as the checker. ``socceraction_amd`` (the product)
never imports it. Parity of the oracle itself is pinned by golden vectors generated
from the reference in the build container (``tests/golden/make_golden.py``).
"""
