"""heat2d_amd.utils"""
