"""heat2d_amd.models"""
