"""Model plugins (the sres.model.<name>.network contract, sres/model/manager.py:93-96)."""
