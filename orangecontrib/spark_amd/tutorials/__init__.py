"""Tutorial workflows (.ows) of the add-on."""
