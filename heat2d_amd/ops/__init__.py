"""heat2d_amd.ops"""
