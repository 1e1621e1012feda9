"""admmtor.eops -- operators (mirror of /root/reference/src/admmtor/eops)."""
