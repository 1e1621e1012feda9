"""admmtor.elayers -- layers (mirror of the ADMMDeconv layer of /root/reference/src/admmtor/elayers)."""
