"""admmtor.eops -- operators (mirror of /root/reference/src/admmtor/eops)."""

# Overlay: when the reference tree is also on sys.path (after this package), its modules that
# this build does not provide (training loop, metrics, data loading, other models) stay
# importable under the same package name; modules present here take precedence.
__path__ = __import__("pkgutil").extend_path(__path__, __name__)
