"""heat2d_amd.parallel"""
