"""admmtor.elayers -- layers (mirror of the ADMMDeconv layer of /root/reference/src/admmtor/elayers)."""

# Overlay: when the reference tree is also on sys.path (after this package), its modules that
# this build does not provide (training loop, metrics, data loading, other models) stay
# importable under the same package name; modules present here take precedence.
__path__ = __import__("pkgutil").extend_path(__path__, __name__)


def __getattr__(name):
    # the reference's elayers/__init__.py re-exports these two (not part of this build); with the
    # reference tree on the path they resolve through the overlay above
    if name in ("LocalAttentionPatch", "PatchProcessor"):
        from . import local_attention_patch
        return getattr(local_attention_patch, name)
    raise AttributeError(name)
