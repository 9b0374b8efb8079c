"""Atomic-SPADL and Atomic-VAEP (reference ``socceraction/atomic``)."""
