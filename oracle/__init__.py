"""TEST INFRASTRUCTURE ONLY: CPU restatements of the reference path (parity checker)."""
