# namespace package (PEP 420 compatible; the reference used pkg_resources.declare_namespace,
# orangecontrib/__init__.py:1-2)
__path__ = __import__("pkgutil").extend_path(__path__, __name__)
