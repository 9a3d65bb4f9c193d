"""CPU oracle for parity tests (test infrastructure; never imported by the
product package ``esslivedata_amd``)."""
