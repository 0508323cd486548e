"""CPU oracle (test infrastructure only): a C++ restatement of the reference apply path.

Never imported by the product package `copycat_amd`."""
