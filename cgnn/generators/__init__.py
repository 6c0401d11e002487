from cgnn_amd.generators import RandomGraphGenerator  # noqa: F401
